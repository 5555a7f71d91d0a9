"""Static check of the DPP64 step-row FMAs in the built library (`fmac_row` in
device_common.hpp).  `v_fmac_f64_dpp ... row_newbcast` is emitted by inline asm, so the compiler's
hazard recognizer does not guard its DPP source: a VALU write of that VGPR in the two instructions
before it would make the broadcast read a stale value.  This disassembles every gfx950 code object
of libgparhip.so (the .hip_fatbin bundles) and fails on any such pair, and on a DPP FMA that opens
a basic block (a predecessor's VALU write could then be adjacent).

    python tools/dpp_hazard_check.py [path/to/libgparhip.so]     -> prints "dpp N hazards 0"
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def code_objects(lib, tmp):
    """gfx950 code objects of every bundle in the library's .hip_fatbin section."""
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib,
                    os.path.join(tmp, "host.so")], check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for i, s in enumerate(starts):
        piece = os.path.join(tmp, f"b{i}.bundle")
        open(piece, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(tmp, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--targets={TARGET}", f"--input={piece}", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def vregs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


def check_listing(text):
    """(number of DPP FMAs, list of hazard descriptions) for one llvm-objdump -d listing."""
    ins = []   # ("L", label) or ("I", text)
    for line in text.splitlines():
        t = line.strip()
        if re.match(r"^[0-9a-f]+ <.*>:$", t):
            ins.append(("L", t))
            continue
        t = t.split("//")[0].strip()
        if not t or t.startswith(";") or t.startswith("Disassembly"):
            continue
        ins.append(("I", t))
    n, bad = 0, []
    for i, (kind, t) in enumerate(ins):
        if kind != "I" or not t.startswith("v_fmac_f64_dpp"):
            continue
        n += 1
        src = vregs(t.split(None, 1)[1].split(",")[1].strip())
        states, j = 0, i - 1
        while j >= 0 and states < 2:
            k2, prev = ins[j]
            if k2 == "L":
                bad.append(f"DPP FMA at a block start: {t}")
                break
            if prev.startswith("s_nop"):
                states += int(prev.split()[1], 0) + 1
            else:
                if prev.startswith("v_") and " " in prev:
                    dst = vregs(prev.split(None, 1)[1].split(",")[0].strip())
                    if dst & src:
                        bad.append(f"{prev} -> {t}")
                states += 1
            j -= 1
    return n, bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpar-at-scale_amd", "libgparhip.so")
    total, hazards = 0, []
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co],
                                 check=True, capture_output=True, text=True).stdout
            n, bad = check_listing(txt)
            total += n
            hazards += bad
    print(f"dpp {total} hazards {len(hazards)}")
    for h in hazards[:20]:
        print("  ", h)
    return 1 if hazards or total == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
