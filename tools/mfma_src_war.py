"""Static scan of compiler-generated MFMA code (hipcc -S output): report every MFMA whose
SrcA / SrcB VGPRs are overwritten by a non-MFMA instruction within N wait states of its issue.

Found in round 5 (profiles/r5/mfma_srcb_war.md): on MI355X a VALU write to an MFMA's SrcB
register in the very next instruction (0 wait states) corrupted that MFMA's operand (the fused
CNN forward's dropout path: 2 % of dOut wrong, bit-exact again once the operand stayed live),
and ROCm 7.2's hazard recognizer does not pad it.

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S kernel.hip -o k.s
    python tools/mfma_src_war.py k.s [max_states=2]
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


def scan(path, max_states=2):
    lines = open(path).read().split("\n")
    fn, hits = None, []
    for i, line in enumerate(lines):
        if re.match(r"^_Z\w+:", line):
            fn = line.split(":")[0]
        t = line.strip()
        if not t.startswith("v_mfma"):
            continue
        ops = t.split(None, 1)[1].split(",")
        src = regs(",".join(ops[1:3]))
        ws = 0
        for k in range(i + 1, min(i + 12, len(lines))):
            u = lines[k].strip()
            if not u or u.startswith(";") or u.startswith("."):
                continue
            if u.startswith("s_nop"):
                ws += int(u.split()[1]) + 1
            else:
                o = u.split(None, 1)
                if len(o) == 2 and not o[0].startswith("v_mfma") and not o[0].startswith("s_"):
                    if regs(o[1].split(",")[0]) & src:
                        hits.append((fn, i + 1, ws, t[:70], u[:60]))
                        break
                ws += 1
            if ws > max_states:
                break
    return hits


if __name__ == "__main__":
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    hits = scan(sys.argv[1], n)
    for fn, ln, ws, a, b in hits:
        print(f"{fn[:60]} line {ln}: {ws} states: {a}  <- {b}")
    print(f"{len(hits)} MFMA source overwrites within {n} wait states")
    sys.exit(1 if hits else 0)
