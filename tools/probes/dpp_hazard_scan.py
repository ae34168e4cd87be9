# ISA check (round 6): no DPP reads a VGPR written by a VALU fewer than 2 wait states before
# (counted in-block, conservative at labels).  Usage: python dpp_hazard_scan.py ipm.s
import re, sys
lines = open(sys.argv[1]).read().split("\n")
def regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m: return set(range(int(m.group(1)), int(m.group(2))+1))
    m = re.match(r"v(\d+)$", op)
    if m: return {int(m.group(1))}
    return set()
hist = []  # list of (kind, dstregs, wait_states)
viol = 0; ndpp = 0
func=None
for i, l in enumerate(lines):
    s = l.strip()
    if re.match(r"^_Z\S+:", l): func = l[:-1]; hist = []
    if not s or s.startswith(";") or s.startswith("."):
        if s.startswith(".LBB") and s.endswith(":"): hist = []  # conservative: reset at labels (fallthrough unknown)
        continue
    parts = s.replace(",", " ").split(); opc = parts[0]; ops = parts[1:]
    if opc == "s_nop":
        n = int(ops[0], 0) + 1
        hist = [(k, d, w + n) for k, d, w in hist]; continue
    if "_dpp" in opc:
        ndpp += 1
        src = regs(ops[1]) if len(ops) > 1 else set()
        for k, d, w in hist:
            if k == "v" and (d & src) and w < 2:
                viol += 1
                if viol < 10: print(func, i + 1, s, "| src written", w, "states before")
    d = regs(ops[0]) if ops and opc.startswith("v_") else set()
    hist = [(k, dd, w + 1) for k, dd, w in hist if w < 8]
    if opc.startswith("v_") and d: hist.append(("v", d, 0))
print("dpp", ndpp, "hazard violations", viol)
