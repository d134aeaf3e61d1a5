"""Generate the two-phase run-keyed merge-join kernels of a TPC-H Q3-shaped join on the CPU
(host tensors stand in for device columns) and write their sources, for offline compile checks:

    python scripts/dev/gen_join_src.py OUT_DIR && hipcc --offload-arch=gfx950 -c OUT_DIR/x.hip
"""
import os
import sys

import numpy as np
import pyarrow as pa

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hyperspace_amd.ops import _lib as NL  # noqa: E402
from hyperspace_amd.exec import jit, jit_runs  # noqa: E402
from hyperspace_amd.exec.device_table import DeviceColumn  # noqa: E402
from hyperspace_amd.exec.encoding import encode, key_runs  # noqa: E402


def agg(kind, terms=()):
    a = NL.AggSpec()
    a.kind, a.nterms = kind, len(terms)
    for t, (c, al, be) in enumerate(terms):
        a.col[t], a.alpha[t], a.beta[t] = c, al, be
    return a


def q3_params(W_groups: int = 1):
    rng = np.random.default_rng(1)
    ok = np.arange(1, 20_001, dtype=np.int64) * 4
    lk = np.repeat(ok, rng.integers(1, 8, len(ok)))
    cl = [DeviceColumn.from_arrow(pa.array(x), "cpu") for x in
          (lk, rng.integers(8000, 10000, len(lk)).astype(np.int32),
           np.round(rng.random(len(lk)) * 1e4, 2), rng.integers(0, 11, len(lk)) / 100.0)]
    cr = [DeviceColumn.from_arrow(pa.array(x), "cpu") for x in
          (ok, rng.integers(8000, 10000, len(ok)).astype(np.int32),
           rng.integers(0, W_groups, len(ok)).astype(np.int32))]
    p = NL.JoinParams()
    for i, c in enumerate(cl):
        p.cols[i] = c.desc()
    for i, c in enumerate(cr):
        p.cols[8 + i] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 9000, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1, 0, 9000, 0.0, None)
    p.nlp, p.npreds = 1, 2
    p.aggs[0] = agg(NL.AK_SUM, [(2, 0.0, 1.0), (3, 1.0, -1.0)])
    p.aggs[1] = agg(NL.AK_COUNT_STAR)
    p.naggs, p.lkey, p.rkey, p.key_is_float = 2, 0, 8, 0
    p.group_col, p.num_groups, p.group_base = 10, W_groups, 0
    allc = dict(enumerate(cl))
    allc.update({8 + i: c for i, c in enumerate(cr)})
    comp = {s: e for s, e in ((s, encode(c)) for s, c in allc.items()) if e is not None}
    comp[0] = key_runs(comp[0])
    return p, comp, (cl, cr)


def main(out):
    os.makedirs(out, exist_ok=True)
    for ng in (1, 3, 200):
        p, comp, keep = q3_params(ng)
        W = jit_runs.tag_width(p)
        NI = jit_runs.RS_ITEMS
        ks = [jit_runs.gen_run_tags2(p, comp, W, jit_runs.RT2_I32), jit_runs.gen_run_scan(p, comp, W, NI)]
        if W == 1 and not (p.group_col >= 8 and p.num_groups > 1):
            ks.append(jit_runs.gen_run_sparse_scan(p, comp))
            # hash walk grouped by the left key (the functionally reduced Q3 GROUP BY)
            from hyperspace_amd.exec import hash_agg as H
            ph, _, _ = q3_params(ng)
            ph.group_col, ph.num_groups = -1, 1
            hk = H.plan_keys([(0, None, keep[0][0], (4, 80_001))], (False, False), False)
            ks.append(jit_runs.gen_run_sparse_scan(ph, comp, hk))
        for k in ks:
            path = os.path.join(out, f"{k.name}_g{ng}.hip")
            with open(path, "w") as f:
                f.write("#include <hip/hip_runtime.h>\n" + k.src)
            print(path)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/jsrc")
