"""Host-side helpers of the kernel wrappers (ops/kernels.py) that need no GPU."""
def test_gather_probe_sample_positions_stay_in_range():
    """The packed-gather probe's sample positions (ops/kernels.py sample_positions) stay in
    [0, n - 2] for table sizes where a float32 linspace would round past the end."""
    import torch
    from hyperspace_amd.ops import kernels as K
    for n in (2, 3, 5, 4097, 16_777_217, 60_000_000, 600_037_902):
        pos = K.sample_positions(n, K.PACKED_SAMPLE, "cpu")
        assert int(pos.min()) >= 0 and int(pos.max()) <= n - 2, n
        assert pos.numel() == min(K.PACKED_SAMPLE, n - 1)
    assert K._random_permutation(torch.randperm(1 << 20))
    assert not K._random_permutation(torch.arange(1 << 20, dtype=torch.int32))
