"""Per-basic-block instruction counts of one kernel in a hipcc -S listing:
   python scripts/asm_blocks.py file.s [kernel-substring]
Prints label, VALU / SALU / LDS / VMEM / branch counts and the branch at the block end."""
import re, sys
path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
blocks, cur = [], None
for l in lines[start:]:
    if l.startswith(".Lfunc_end"):
        break
    m = re.match(r"^(\.LBB\S+|_Z\S+|; %bb\.\d+):?", l)
    if m:
        cur = {"label": m.group(1).rstrip(":"), "v": 0, "s": 0, "ds": 0, "vm": 0, "br": "", "n": 0, "other": ""}
        blocks.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith(".") or cur is None:
        continue
    op = t.split()[0]
    cur["n"] += 1
    if op.startswith("v_"):
        cur["v"] += 1
    elif op.startswith("ds_"):
        cur["ds"] += 1
    elif op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        cur["vm"] += 1
    elif op.startswith("s_cbranch") or op == "s_branch":
        cur["br"] = t
    elif op.startswith("s_"):
        cur["s"] += 1
for b in blocks:
    print(f"{b['label']:24s} v{b['v']:4d} s{b['s']:4d} ds{b['ds']:3d} vm{b['vm']:3d}  {b['br']}")
print("total v", sum(b["v"] for b in blocks), "s", sum(b["s"] for b in blocks))
