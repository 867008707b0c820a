"""Per-kernel register / occupancy / LDS summary of one HIP source, from
hipcc -Rpass-analysis=kernel-resource-usage (compile only, no GPU).

    python tools/kernel_resources.py ska-sdp-func-radler_amd/csrc/hip/fft_fast.hip [filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-ffp-contract=off", f"-I{ROOT}/include",
           f"-I{ROOT}/ska-sdp-func-radler_amd/csrc/hip", "-c", src, "-o", "/tmp/_kr.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill|"
                      r"SGPRs Spill|LDS Size \[bytes/block\]|SGPRs): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                           capture_output=True, text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        if filt and filt not in n:
            continue
        print(f"{r.get('VGPRs', 0):4d} v {r.get('AGPRs', 0):3d} a "
              f"occ {r.get('Occupancy [waves/SIMD]', 0)} "
              f"spill {r.get('VGPRs Spill', 0):3d} lds {r.get('LDS Size [bytes/block]', 0):6d}"
              f"  {n[:150]}")


if __name__ == "__main__":
    main()
