"""Static VALU instruction mix per kernel of libzkp's gfx950 code object.

Classifies each VALU instruction as FAST (issues every 2 SIMD cycles per wave64:
plain 2-operand 32-bit ops) or SLOW (every 4 cycles: carry in/out, multiplies,
3-operand, 64-bit and SGPR-reading ops), per tests/native/ubench_valu.hip
(profiles/r02_ubench_valu.txt). Writes a JSON map kernel symbol -> counts and
slow_frac. The kernels are straight-line unrolled bodies, so the static mix is
a close stand-in for the dynamic one.
Usage: python3 scripts/isa_mix.py [kernels.o] > profiles/r02_isa_mix.json
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_or_b32", "v_and_b32", "v_mov_b32",
        "v_lshlrev_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_not_b32", "v_add_u16", "v_sub_u16"}


def disasm(obj):
    d = tempfile.mkdtemp()
    fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
    subprocess.check_call(["objcopy", "--dump-section", f".hip_fatbin={fb}", obj])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], text=True)


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return dict(zip(names, out))


def main(objs):
    txt = "\n".join(disasm(o) for o in objs)
    cur, per = None, collections.defaultdict(collections.Counter)
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            continue
        m = re.match(r"^\s+(v_[a-z0-9_]+)", line)
        if cur and m:
            op = re.sub(r"_e(32|64)$|_sdwa$|_dpp$", "", m.group(1))
            per[cur]["fast" if op in FAST else "slow"] += 1
            per[cur]["op:" + op] += 1
    names = demangle(list(per))
    res = {}
    for k, c in per.items():
        tot = c["fast"] + c["slow"]
        top = sorted(((v, o[3:]) for o, v in c.items() if o.startswith("op:")), reverse=True)[:8]
        res[names[k]] = {"valu_static": tot, "fast": c["fast"], "slow": c["slow"],
                         "slow_frac": round(c["slow"] / tot, 4) if tot else None, "top_ops": top}
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    build = os.path.join(os.path.dirname(__file__), "..", "zk_stark_project_amd", "csrc", "build")
    main(sys.argv[1:] or [os.path.join(build, "kernels.o"), os.path.join(build, "ntt.o")])
