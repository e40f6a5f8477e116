"""Estimated VALU issue cycles per basic block of one kernel in a hipcc -S listing,
with gfx950 per-instruction costs measured by scripts/micro/valu_rate*.hip
(profiles/r3_valu_rate.txt): 2 cycles for the simple VOP2 ALU ops and v_bitop3 with
VGPR / literal / inline operands; 4 cycles for everything else and for ANY
instruction that reads an SGPR (constant-bus) operand.
   python scripts/asm_cost.py file.s [kernel-substring] [--all]"""
import re
import sys

FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshrrev_b32",
        "v_lshlrev_b32", "v_ashrrev_i32", "v_mov_b32", "v_bitop3_b32", "v_not_b32", "v_cndmask_b32", "v_min_u32",
        "v_max_u32", "v_min_i32", "v_max_i32", "v_add_co_u32", "v_sub_co_u32", "v_addc_co_u32", "v_subb_co_u32",
        "v_subbrev_co_u32", "v_bitop3_b16", "v_xnor_b32"}
path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
blocks, cur = [], None
sgpr = re.compile(r"(?<![\w\[])(s\d+|s\[\d+:\d+\]|vcc|exec|m0)(?![\w])")
for l in lines[start:]:
    if l.startswith(".Lfunc_end"):
        break
    m = re.match(r"^(\.LBB\S+|_Z\S+|; %bb\.\d+):?", l)
    if m:
        cur = {"label": m.group(1).rstrip(":"), "cyc": 0, "v": 0, "slow": {}, "br": ""}
        blocks.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith(".") or cur is None:
        continue
    op = t.split()[0]
    if op.startswith("s_cbranch") or op == "s_branch":
        cur["br"] = t.split(";")[0]
    if not op.startswith("v_"):
        continue
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    args = t[len(op):].split(";")[0]
    # implicit vcc of e32 cndmask / carry ops does not count as a constant-bus operand here
    reads_s = bool(sgpr.search(args.split(",", 1)[1] if "," in args else "")) and not (
        base in ("v_cndmask_b32", "v_addc_co_u32", "v_subb_co_u32", "v_subbrev_co_u32") and op.endswith("e32"))
    c = 2 if (base in FAST and not reads_s) else 4
    if base.startswith("v_cmp"):
        c = 4
    cur["cyc"] += c
    cur["v"] += 1
    if c == 4:
        key = base + (" [s]" if reads_s else "")
        cur["slow"][key] = cur["slow"].get(key, 0) + 1
for b in blocks:
    if b["v"] or "--all" in sys.argv:
        top = ", ".join(f"{k} x{n}" for k, n in sorted(b["slow"].items(), key=lambda kv: -kv[1])[:6])
        print(f"{b['label']:14s} v{b['v']:4d} cyc{b['cyc']:5d}  {b['br'][:30]:30s} {top}")
print("total v", sum(b["v"] for b in blocks), "cycles", sum(b["cyc"] for b in blocks))
