# ISA check (round 6): every half-row DPP move (bank_mask:0x3) must be followed by its bank_mask:0xc
# partner on the same destination before anything reads or writes that register.  Usage: python dpp_pair_scan.py ipm.s
# (the .s from hipcc --cuda-device-only -S).
import re, sys
lines = open(sys.argv[1]).read().split("\n")
def regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m: return set(range(int(m.group(1)), int(m.group(2))+1))
    m = re.match(r"v(\d+)$", op)
    if m: return {int(m.group(1))}
    return set()
bad = 0; n = 0; kinds = {}
func = None
for i, l in enumerate(lines):
    if re.match(r"^_Z\S+:", l): func = l[:-1]
    if "bank_mask:0x3 " not in l: continue
    n += 1
    ins = l.split()
    dst = regs(ins[1].rstrip(","))
    m = re.search(r"row_newbcast:(\d+)", l); lane = int(m.group(1))
    # walk forward
    j = i + 1; ok = None
    while j < len(lines):
        s = lines[j].strip()
        j += 1
        if not s or s.startswith(";") or s.startswith(".") : 
            if s.startswith(".LBB") or (s.startswith(".") and s.endswith(":")):
                ok = "label:" + s; break
            continue
        if s.startswith("s_cbranch") or s.startswith("s_branch") or s.startswith("s_setpc"):
            ok = "branch:" + s; break
        parts = s.replace(",", " ").split()
        opc = parts[0]; ops = parts[1:]
        d = regs(ops[0]) if ops else set()
        srcs = set()
        for o in ops[1:]: srcs |= regs(o)
        if "bank_mask:0xc" in s and d == dst:
            ok = "pair"; break
        if dst & srcs:
            ok = "READ-before-pair: " + s; break
        if dst & d and not opc.startswith(("global_store","buffer_store","scratch_store","ds_write","flat_store")):
            ok = "WRITE-before-pair: " + s; break
        if opc.startswith(("s_and_saveexec","s_or_saveexec","s_mov_b64 exec","s_or_b64 exec","s_andn2_b64 exec","s_xor_b64 exec","s_and_b64 exec")) or " exec" in s and opc.startswith("s_"):
            kinds["exec-change-between"] = kinds.get("exec-change-between", 0) + 1
    k = ok.split(":")[0] if ok else "eof"
    kinds[k] = kinds.get(k, 0) + 1
    if k != "pair":
        bad += 1
        if bad <= 12: print(func, i+1, l.strip(), "->", ok)
print(n, kinds)
