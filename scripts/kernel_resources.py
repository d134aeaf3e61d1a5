#!/usr/bin/env python
"""Per-kernel VGPR / AGPR / spill / occupancy table for a .hip file (gfx950), from the compiler's
kernel-resource-usage remarks.  Usage: python scripts/kernel_resources.py csrc/kernels/join.hip"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]


def main(paths):
    for path in paths:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-munsafe-fp-atomics", "-c", path, "-o", "/dev/null",
               "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, capture_output=True, text=True).stderr
        cur = None
        rows = []
        for line in out.splitlines():
            m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
            if not m:
                continue
            k, v = m.group(1).strip(), m.group(2).strip()
            if k == "Function Name":
                cur = {"name": subprocess.run(["c++filt", v], capture_output=True,
                                              text=True).stdout.strip()}
                rows.append(cur)
            elif cur is not None:
                cur[k] = v
        print(path)
        for r in rows:
            print(f"  {r['name'][:60]:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} "
                  f"occ={r.get('Occupancy [waves/SIMD]','?'):>2} "
                  f"vspill={r.get('VGPRs Spill','?')} sspill={r.get('SGPRs Spill','?')} "
                  f"lds={r.get('LDS Size [bytes/block]','?')}")


if __name__ == "__main__":
    main(sys.argv[1:])
