"""Static check of hand-scheduled MFMA code: report any non-MFMA instruction that overwrites a
VGPR / AGPR an inline-asm MFMA reads (SrcA / SrcB / SrcC), or touches its destination, within
N instructions after that MFMA.

The compiler does not know an inline-asm MFMA still reads its operands after issue, so it may
allocate a VALU result into them at once (seen in the persistent LSTM forward: a
v_accvgpr_read into SrcA one instruction after the MFMA -> wrong h). Usage:

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S kernel.hip -o k.s
    python tools/mfma_war.py k.s [window=4]
"""
import re
import sys


def regs(text):
    out = set()
    for m in re.finditer(r"\b([va])\[(\d+):(\d+)\]", text):
        out.update(f"{m.group(1)}{r}" for r in range(int(m.group(2)), int(m.group(3)) + 1))
    for m in re.finditer(r"\b([va])(\d+)\b", text):
        out.add(m.group(1) + m.group(2))
    return out


def check(path, window=4):
    src = open(path).read()
    bad = 0
    for fm in re.finditer(r"^(_Z\w+):", src, re.M):
        name = fm.group(1)
        end = src.find(".Lfunc_end", fm.end())
        lines = [ln.split(";")[0].strip() for ln in src[fm.end():end].split("\n")]
        lines = [ln for ln in lines if ln and not ln.startswith(".") and not ln.endswith(":")]
        recent = []
        for k, ln in enumerate(lines):
            parts = ln.split(None, 1)
            op = parts[0]
            if len(parts) < 2 or op.startswith(("s_", "ds_read", "global_load", "buffer_load")):
                continue  # scalar ops; loads write their destination long after issue
            dst = regs(parts[1].split(",")[0])
            used = regs(",".join(parts[1].split(",")[1:]))
            for mk, srcs, mdst in recent:
                if k - mk <= window and "mfma" not in op and (dst & srcs or (dst | used) & mdst):
                    bad += 1
                    print(f"{name[:60]}: +{k - mk}: {lines[mk]}  ||  {ln}")
            if "mfma" in op:
                ops = parts[1].split(",")
                recent = (recent + [(k, regs(",".join(ops[1:])), regs(ops[0]))])[-8:]
    print(f"{path}: {bad} overwrite(s) of MFMA source registers within {window} instructions")
    return bad


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4) else 0)
