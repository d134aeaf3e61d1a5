"""``parallel.shuffle.exchange`` on device tensors (the packed all-to-all's device path defers a
batch until its counts copy lands: ``RowExchange._add_device``).  Single process: the exchange is
a local copy, so every row comes back, grouped by destination in source order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_shuffle_exchange_on_device(device):
    import torch
    from hyperspace_amd.parallel.shuffle import exchange
    rng = np.random.default_rng(3)
    n = 10_000
    a = torch.from_numpy(rng.integers(-1 << 40, 1 << 40, n)).to(device)
    b = torch.from_numpy(rng.random(n)).to(device)
    dest = torch.zeros(n, dtype=torch.int64, device=device)
    (ra, none, rb), counts = exchange([a, None, b], dest, 1)
    assert none is None
    assert ra.is_cuda and rb.is_cuda
    assert counts.tolist() == [n]
    assert torch.equal(ra, a) and torch.equal(rb, b)
