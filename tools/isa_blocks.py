"""VALU / SALU / memory instructions per basic block of one kernel in a gfx950 assembly listing
(hipcc -S --cuda-device-only), with the compiler's loop annotations -- the static half of the
blend's VALU account (tools/valu_account.py).
usage: python tools/isa_blocks.py listing.s 'k_drawILb0ELb0ELb0E'"""
import re
import sys

src, key = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\w*" + key + r"\w*:", ln))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur, blocks = ["entry", "", 0, 0, 0], []
for ln in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?(.*)", ln)
    if m:
        blocks.append(cur)
        cur = [m.group(1), m.group(2).strip(), 0, 0, 0]
        continue
    t = ln.strip().split()
    if not t or t[0].startswith(";") or t[0].startswith("."):
        continue
    op = t[0]
    if op.startswith("v_"):
        cur[2] += 1
    elif op.startswith("s_"):
        cur[3] += 1
    elif op.startswith(("ds_", "global_", "buffer_", "flat_")):
        cur[4] += 1
blocks.append(cur)
print(f"{lines[start].split(':')[0]}: {len(blocks)} blocks, {sum(b[2] for b in blocks)} VALU in all")
for b in blocks:
    if b[2] or b[4]:
        print(f"{b[0]:14s} valu={b[2]:3d} salu={b[3]:3d} mem={b[4]:2d}  {b[1][:70]}")
