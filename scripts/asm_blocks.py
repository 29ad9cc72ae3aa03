"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (gfx950).

    python scripts/asm_blocks.py file.s <mangled-kernel-name> [--min 20]

Prints each block with >= --min instructions: MFMA, VALU (exp / cvt_pk / mov separately), SALU,
LDS, global/buffer, waitcnt, and the block's successors -- the quick way to see where a kernel's
VALU goes before a PMC run."""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 20
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur, label = [], [], "entry"
for l in lines[start + 1:end]:
    s = l.strip()
    if re.match(r"^\.?L\w+:", s) or re.match(r"^\.LBB\w+:", s):
        blocks.append((label, cur))
        label, cur = s.split(":")[0], []
        continue
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur.append(s.split(";")[0].strip())
blocks.append((label, cur))


def cat(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_exp"):
        return "exp"
    if op.startswith("v_cvt_pk_bf16"):
        return "cvtpk"
    if op.startswith("v_mov") or op.startswith("v_accvgpr"):
        return "vmov"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith("v_cmp"):
        return "vcmp"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("buffer_") or op.startswith("global_"):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "br"
    if op.startswith("s_"):
        return "salu"
    return "other"


if "--dump" in sys.argv:  # opcode histogram (or the text with --text) of one block
    want = sys.argv[sys.argv.index("--dump") + 1]
    for label, ins in blocks:
        if label == want:
            if "--text" in sys.argv:
                print("\n".join(ins))
            else:
                from collections import Counter
                for op, n in Counter(i.split()[0] for i in ins).most_common():
                    print(f"{n:5d} {op}")
    sys.exit(0)

keys = ["mfma", "exp", "valu", "vmov", "cvtpk", "cndmask", "vcmp", "lds", "vmem", "wait", "salu", "br"]
print("block".ljust(14), " ".join(k.rjust(6) for k in keys), " total")
tot = {k: 0 for k in keys}
for label, ins in blocks:
    c = {k: 0 for k in keys}
    for i in ins:
        k = cat(i)
        if k in c:
            c[k] += 1
    for k in keys:
        tot[k] += c[k]
    if len(ins) >= mn:
        br = [i for i in ins if cat(i) == "br"]
        print(label.ljust(14), " ".join(str(c[k]).rjust(6) for k in keys), str(len(ins)).rjust(6), " ", "; ".join(br)[:60])
print("TOTAL".ljust(14), " ".join(str(tot[k]).rjust(6) for k in keys))
