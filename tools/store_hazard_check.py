#!/usr/bin/env python3
"""Scan gfx950 assembly for the store-data WAR hazard behind the bf16 quad-epilogue nondeterminism:
a VMEM store of more than 8 bytes (buffer/global/flat _dwordx3/_dwordx4, _b96/_b128) whose data VGPRs
are overwritten by a VALU instruction with no wait state in between.  The store reads its data some
cycles after issue; the compiler's hazard recognizer pads such a write with an s_nop inside one basic
block, but the quad epilogue's `if (p.out_h2)` diamond put the overwrite after a block boundary
(store in one block, the join label, then the write) with nothing in between, and the stored dword
came out with the NEXT value at random (tools/lbbench.py WHERE=1: always the store's first dword).
usage: store_hazard_check.py file.s [...]   (hipcc --cuda-device-only -S)
       store_hazard_check.py --lib libtcx.so   (every gfx950 code object in the library, disassembled)
exit 1 when any is found"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"

STORE = re.compile(r"^\s+(buffer|global|flat)_store_(dwordx3|dwordx4|b96|b128)\s+(v\[(\d+):(\d+)\]|v\d+),?\s*(v\[(\d+):(\d+)\]|v\d+)?")
INSTR = re.compile(r"^\s+([a-z_0-9]+)")


def vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def data_regs(line, kind):
    ops = [o.strip() for o in line.split(None, 1)[1].split(",")]
    # buffer_store: data, vaddr, srsrc, soffset; global_store: vaddr, data, saddr; flat_store: vaddr, data
    return vregs(ops[0] if kind == "buffer" else ops[1])


def dst_regs(line):
    parts = line.split(None, 1)
    if len(parts) < 2:
        return set()
    return vregs(parts[1].split(",")[0].strip())


WAIT_STATES = 2  # VALU write of a >8-byte VMEM store's data VGPRs: wait states required on gfx940+ (gfx950)
ADDR = re.compile(r"//\s*([0-9A-Fa-f]{8,}):")
OBJ_TGT = re.compile(r"<(_Z[^+>\s]+)\+0x([0-9a-f]+)>")
FUNC = re.compile(r"^([0-9a-f]+) <(_Z[^>\s]+)>:")


def _index(lines):
    """instruction line -> address (objdump listings) and label / address -> line of the target"""
    addr_line, label_line, func_addr = {}, {}, {}
    for i, l in enumerate(lines):
        m = FUNC.match(l)
        if m:
            func_addr[m.group(2)] = int(m.group(1), 16)
            continue
        m = re.match(r"^(\.L[A-Za-z0-9_$.]+):", l)
        if m:
            label_line[m.group(1)] = i
            continue
        m = ADDR.search(l)
        if m and INSTR.match(l):
            addr_line[int(m.group(1), 16)] = i
    return addr_line, label_line, func_addr


def _branch_target(l, addr_line, label_line, func_addr):
    m = OBJ_TGT.search(l)
    if m and m.group(1) in func_addr:
        return addr_line.get(func_addr[m.group(1)] + int(m.group(2), 16))
    parts = l.split(None, 1)
    if len(parts) > 1:
        tok = parts[1].split("//")[0].strip().split(",")[0].strip()
        if tok in label_line:
            return label_line[tok]
    return None


def _next_instr(lines, j):
    while j < len(lines):
        l = lines[j]
        if l.startswith(".Lfunc_end") or FUNC.match(l):
            return None
        if INSTR.match(l) and not l.strip().startswith(";") and not l.strip().startswith("."):
            return j
        j += 1
    return None


def scan(path):
    """every >8-byte VMEM store whose data VGPRs a VALU instruction writes within WAIT_STATES wait
    states on ANY path: the fall-through, the target of an s_branch and both sides of an s_cbranch
    (each instruction in between is one wait state, s_nop N is N + 1)"""
    lines = open(path).read().split("\n")
    addr_line, label_line, func_addr = _index(lines)
    fn = "?"
    found = 0
    for i, l in enumerate(lines):
        m = re.match(r"^(?:[0-9a-f]+ <)?(_Z[^>\s]+)>?:", l)
        if m:
            fn = m.group(1)
        sm = STORE.match(l)
        if not sm:
            continue
        regs = data_regs(l, sm.group(1))
        work = [(i + 1, 0)]
        seen = set()
        hit = None
        while work and hit is None:
            j0, ws = work.pop()
            j = _next_instr(lines, j0)
            while j is not None and ws < WAIT_STATES:
                if (j, ws) in seen:
                    break
                seen.add((j, ws))
                nxt = lines[j]
                op = INSTR.match(nxt).group(1)
                if op.startswith("v_") and not op.startswith("v_cmp") and dst_regs(nxt) & regs:
                    hit = (nxt, ws)
                    break
                if op == "s_nop":
                    arg = nxt.split(None, 1)[1].split("//")[0].strip() if len(nxt.split(None, 1)) > 1 else "0"
                    ws += int(arg, 0) + 1
                else:
                    ws += 1
                if op == "s_endpgm":
                    break
                if op.startswith("s_branch") or op.startswith("s_cbranch"):
                    t = _branch_target(nxt, addr_line, label_line, func_addr)
                    if t is not None:
                        work.append((t, ws))
                    if op.startswith("s_branch"):
                        break
                j = _next_instr(lines, j + 1)
        if hit is not None:
            found += 1
            print(f"{path}:{i + 1}: {fn[:90]}\n    {l.strip()}\n    {hit[0].strip()}   <- overwrites store data, "
                  f"{hit[1]} wait state(s)")
    return found


def lib_listings(so, tmp):
    """disassemble each gfx950 code object of the library's .hip_fatbin (one offload bundle per
    translation unit, concatenated by the link)"""
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", so, os.path.join(tmp, "so")],
                   check=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = []
    i = data.find(magic)
    while i >= 0:
        offs.append(i)
        i = data.find(magic, i + 1)
    out = []
    for k, o in enumerate(offs):
        piece = os.path.join(tmp, f"b{k}")
        with open(piece, "wb") as fh:
            fh.write(data[o:offs[k + 1] if k + 1 < len(offs) else len(data)])
        co = os.path.join(tmp, f"b{k}.co")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={piece}", f"--output={co}"], check=True)
        dis = os.path.join(tmp, f"b{k}.s")
        with open(dis, "w") as fh:
            subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, stdout=fh)
        out.append(dis)
    return out


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--lib":
        with tempfile.TemporaryDirectory() as tmp:
            files = lib_listings(sys.argv[2], tmp)
            n = sum(scan(p) for p in files)
            print(f"{len(files)} code objects scanned")
    else:
        n = sum(scan(p) for p in sys.argv[1:])
    print(f"{n} hazard(s)")
    sys.exit(1 if n else 0)
