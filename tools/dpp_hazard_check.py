"""Static check of the DPP64 step-row FMAs in the built library (`fmac_row` in
device_common.hpp).  `v_fmac_f64_dpp ... row_newbcast` is emitted by inline asm, so the compiler's
hazard recognizer does not guard its DPP source: a VALU write of that VGPR in the two instructions
before it would make the broadcast read a stale value.  This disassembles every gfx950 code object
of libgparhip.so (the .hip_fatbin bundles) and fails on any such pair along every control-flow
predecessor: branch targets are resolved from llvm-objdump --symbolize-operands, so a DPP FMA at a
loop header or join is checked against the tail of each block that branches there as well as the
fall-through.

It also checks every wide (x3 / x4) VMEM store against a VALU write of its data registers in the
next instruction (check_store_listing).

    python tools/dpp_hazard_check.py [path/to/libgparhip.so]  -> "dpp N hazards 0 wide_stores S"
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


UNCOND = ("s_branch", "s_endpgm", "s_setpc_b64")


def _functions(text):
    """llvm-objdump --symbolize-operands listing -> {function: [("L", label) | ("I", text)]}.
    Branch targets appear as "<Ln>:" lines (numbered per function), branch operands as "Ln"."""
    funcs, cur = {}, None
    for line in text.splitlines():
        t = line.strip()
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", t)
        if m:
            if re.fullmatch(r"L\d+", m.group(1)) and cur is not None:
                funcs[cur].append(("L", m.group(1)))
            else:
                cur = m.group(1)
                funcs[cur] = []
            continue
        t = t.split("//")[0].strip()
        if not t or t.startswith(";") or t.startswith("Disassembly") or cur is None:
            continue
        funcs[cur].append(("I", t))
    return funcs


def check_listing(text):
    """(number of DPP FMAs, list of hazard descriptions) for one llvm-objdump -d
    --symbolize-operands listing.  For each DPP FMA the two wait states before it are searched
    along EVERY control-flow predecessor: at a branch-target label, both the fall-through from the
    instructions laid out before it (unless those end in an unconditional branch) and the tail of
    every block that branches there (the branch itself counted as no wait state)."""
    n, bad = 0, []
    for fname, ins in _functions(text).items():
        label_at = {t: i for i, (k, t) in enumerate(ins) if k == "L"}
        preds = {}   # label -> indices of the branches that target it
        for i, (k, t) in enumerate(ins):
            if k == "I" and t.startswith(("s_branch", "s_cbranch")):
                parts = t.split()
                if len(parts) > 1 and parts[1] in label_at:
                    preds.setdefault(parts[1], []).append(i)

        def walk(j, states, src, dpp, seen):
            """Hazards for a DPP FMA reading src, walking back from index j with `states` wait
            states already between it and the DPP FMA."""
            out = []
            while j >= 0 and states < 2:
                if (j, states) in seen:
                    return out
                seen.add((j, states))
                k2, prev = ins[j]
                if k2 == "L":
                    for b in preds.get(prev, []):
                        out += walk(b - 1, states, src, dpp, seen)
                    if j > 0 and ins[j - 1][0] == "I" and ins[j - 1][1].startswith(UNCOND):
                        return out   # no fall-through into this block
                    j -= 1
                    continue
                if prev.startswith("s_nop"):
                    states += int(prev.split()[1], 0) + 1
                else:
                    if prev.startswith("v_") and " " in prev:
                        dst = vregs(prev.split(None, 1)[1].split(",")[0].strip())
                        if dst & src:
                            out.append(f"{fname}: {prev} -> {dpp}")
                    states += 1
                j -= 1
            return out

        for i, (kind, t) in enumerate(ins):
            if kind != "I" or not t.startswith("v_fmac_f64_dpp"):
                continue
            n += 1
            src = vregs(t.split(None, 1)[1].split(",")[1].strip())
            if i > 0 and ins[i - 1][0] == "L" and ins[i - 1][1] not in preds:
                bad.append(f"{fname}: DPP FMA after an unresolved label: {t}")
            bad += walk(i - 1, 0, src, t, set())
    return n, bad


STORE_WIDE = re.compile(r"^(global|buffer|flat|scratch)_store_dwordx[34]\b")


def check_store_listing(text):
    """(number of wide stores, hazards): a VMEM store of more than 64 bits of data reads its data
    VGPRs after issue, so a VALU write of them in the very next instruction (no wait state) can
    change what is stored.  hipcc pads its own stores; an inline-asm store hides this from it (the
    round-5 gains fast path's first version: asm record stores, wrong records on some waves of
    some launches).  Checked along the laid-out successor (labels fall through)."""
    n, bad = 0, []
    for fname, ins in _functions(text).items():
        for i, (kind, t) in enumerate(ins):
            if kind != "I" or not STORE_WIDE.match(t):
                continue
            n += 1
            ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
            data = vregs(ops[1]) if len(ops) > 1 else set()
            j = i + 1
            while j < len(ins) and ins[j][0] == "L":
                j += 1
            if j >= len(ins):
                continue
            nxt = ins[j][1]
            if nxt.startswith("v_") and " " in nxt:
                dst = vregs(nxt.split(None, 1)[1].split(",")[0].strip())
                if dst & data:
                    bad.append(f"{fname}: {t} -> {nxt}")
    return n, bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpar-at-scale_amd", "libgparhip.so")
    total, hazards, stores = 0, [], 0
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands",
                                  "--mcpu=gfx950", co],
                                 check=True, capture_output=True, text=True).stdout
            n, bad = check_listing(txt)
            total += n
            hazards += bad
            ns, sbad = check_store_listing(txt)
            stores += ns
            hazards += sbad
    print(f"dpp {total} hazards {len(hazards)} wide_stores {stores}")
    for h in hazards[:20]:
        print("  ", h)
    return 1 if hazards or total == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
