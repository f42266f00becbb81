#!/usr/bin/env python3
"""Static check of a compiled kernel (.s from hipcc --cuda-device-only -S) for the hazard that
corrupted k_conv3m under concurrent kernels (r04_n): an MFMA whose accumulator is moved to a new
register (D != C) leaves its old SrcC register free, and a later ds_read / buffer_load writes that
register while the MFMA - queued behind other waves' MFMAs on the matrix pipe - may not have read it
yet.  Reports every load whose destination overlaps the SrcC (or SrcA / SrcB) registers of an MFMA
issued within the last WINDOW MFMAs of the same basic block stream.
usage: mfma_war_check.py file.s kernel_symbol [window]"""
import re
import sys


def regs(tok):
    m = re.match(r"[va]\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1)), tok[0]
    m = re.match(r"([va])(\d+)$", tok)
    if m:
        return {int(m.group(2))}, m.group(1)
    return set(), None


def main() -> int:
    path, sym = sys.argv[1], sys.argv[2]
    window = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    recent = []  # (line, kind, regfile, regs) of the last `window` MFMAs' sources
    hits = {"C": 0, "AB": 0}
    for i in range(start, end):
        t = lines[i].strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        args = [a.strip() for a in t[len(op):].split(",")]
        if op.startswith("v_mfma"):
            d, df = regs(args[0])
            a, af = regs(args[1])
            b, bf = regs(args[2])
            c, cf = regs(args[3])
            ent = [(i, "AB", af, a), (i, "AB", bf, b)]
            if c != d:
                ent.append((i, "C", cf, c))
            recent.append(ent)
            recent = recent[-window:]
        elif op.startswith("ds_read") or op.startswith("buffer_load") or op.startswith("global_load"):
            if " lds" in t:
                continue
            dst, dfile = regs(args[0])
            for ent in recent:
                for (li, kind, rf, rs) in ent:
                    if rf == dfile and rs & dst:
                        hits[kind] += 1
                        if hits[kind] <= 5:
                            print(f"{kind}: line {i - start}: {t}  overwrites a source of line {li - start}: {lines[li].strip()}")
    print(f"{sym}: loads overwriting a recent MFMA's moved SrcC: {hits['C']}, its SrcA/SrcB: {hits['AB']}")
    return 1 if hits["C"] else 0


if __name__ == "__main__":
    raise SystemExit(main())
