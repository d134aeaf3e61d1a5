#!/usr/bin/env python
"""Device timeline of the bench's timed steps from a gpu.sh `benchtrace` kernel trace: finds the
longest stretch of the headline's query kernels (two-phase join tags / bits scan, Q6 scan), then
reports the stretch's wall time, how much of it the GPU had any kernel running (interval
union), the idle gaps, and per-kernel counts and mean durations.

    python scripts/diag/step_timeline.py gpurun_out/X_bench_ktrace.csv [steps]
"""
import collections
import csv
import sys

HOT = ("hs_jit_run_tags2", "hs_jit_run_bits_scan", "hs_jit_scan_agg")


def main():
    rows = [(r["name"], int(r["start"]), int(r["end"]), r["queue"])
            for r in csv.DictReader(open(sys.argv[1]))]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows.sort(key=lambda x: x[1])
    # the timed run: the densest window of `steps` bits-scan launches with no join-index or
    # top-k kernel inside (those belong to the side runs)
    idx = [i for i, r in enumerate(rows) if r[0].startswith("hs_jit_run_bits_scan")]
    best = None
    for a in range(len(idx) - steps + 1):
        lo, hi = idx[a], idx[a + steps - 1]
        if any(r[0].startswith(("hs_jit_join_index", "hs_jit_run_bits_topk"))
               for r in rows[lo:hi]):
            continue
        span = rows[hi][1] - rows[lo][1]
        if best is None or span < best[2]:
            best = (lo, hi, span)
    if best is None:
        sys.exit("no timed stretch found")
    lo, hi, _ = best
    # widen to the first tags kernel before and the scans around
    while lo > 0 and rows[lo - 1][0].startswith(HOT + ("hs_agg_final",)):
        lo -= 1
    seg = rows[lo:hi + 1]
    t0, t1 = seg[0][1], max(r[2] for r in seg)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for _, s, e, _ in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = t1 - t0
    print(f"timed stretch: {len(seg)} kernels, wall {wall / 1e6:.3f} ms "
          f"({wall / 1e3 / steps:.1f} us per step over {steps} steps)")
    print(f"GPU busy (union) {busy / 1e6:.3f} ms = {100 * busy / wall:.1f}%; "
          f"idle gaps: {len(gaps)}, total {sum(gaps) / 1e6:.3f} ms, "
          f"largest {max(gaps, default=0) / 1e3:.1f} us")
    per = collections.defaultdict(list)
    for n, s, e, q in seg:
        per[n.split("(")[0]].append(e - s)
    print(f"{'kernel':44s} {'calls':>6s} {'mean us':>9s} {'per step us':>12s}")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:44]:44s} {len(d):6d} {sum(d) / len(d) / 1e3:9.1f} "
              f"{sum(d) / steps / 1e3:12.1f}")
    qs = collections.Counter(q for _, _, _, q in seg)
    print("queues:", dict(qs))


if __name__ == "__main__":
    main()
