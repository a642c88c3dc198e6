#!/usr/bin/env python3
"""Per-kernel gfx950 resource usage of the HIP sources (VGPRs, scratch, spills,
LDS, occupancy) from the compiler's kernel-resource-usage remarks; prints every
kernel, flags those with private (scratch) memory. Usage (from the repo root):
    python scripts/kernel_resources.py [out.txt]
Device-only compile of each .hip TU, same flags as csrc/Makefile."""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zk_stark_project_amd", "csrc")
TUS = ["kernels.hip", "merkle.hip", "ntt.hip"]


def remarks(tu):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-c",
           os.path.join(CSRC, tu), "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr)
    rows, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {"tu": tu}
            continue
        m = re.search(r"remark: +([A-Za-z \[\]/]+): (\S+)", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    for tool in ("/opt/rocm/lib/llvm/bin/llvm-cxxfilt", "c++filt"):
        try:
            r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
        except OSError:
            continue
        if r.returncode == 0:
            return r.stdout.splitlines()
    return names


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main():
    with cf.ThreadPoolExecutor(len(TUS)) as ex:
        rows = {}
        for part in ex.map(remarks, TUS):
            rows.update(part)
    names = list(rows)
    pretty = dict(zip(names, demangle(names)))
    out = []
    flagged = 0
    for k in sorted(names, key=lambda n: (rows[n]["tu"], pretty[n])):
        v = rows[k]
        scratch = int(v.get("ScratchSize [bytes/lane]", "0"))
        spill = int(v.get("VGPRs Spill", "0")) + int(v.get("SGPRs Spill", "0"))
        flag = "  <-- scratch" if scratch or spill else ""
        flagged += bool(flag)
        out.append(f"{v['tu']:12s} vgpr={v.get('VGPRs', '?'):>4s} scratch={scratch:4d} spill={spill:3d} "
                   f"lds={v.get('LDS Size [bytes/block]', '?'):>6s} occ={v.get('Occupancy [waves/SIMD]', '?'):>2s} "
                   f"{short(pretty[k])}{flag}")
    out.append(f"{len(names)} kernels, {flagged} with scratch or spills")
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
