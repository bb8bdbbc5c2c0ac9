"""Per-basic-block instruction census of one kernel in a hipcc -S file (which blocks hold the MFMAs, and how much
VALU / LDS / wait traffic sits beside them).  usage: python tools/isa_blocks.py file.s kernel_substring"""
import sys
from collections import Counter

src, key = sys.argv[1], sys.argv[2]
s = open(src).read()
start = [i for i in range(len(s)) if s.startswith(key, i)]
i = s.index(":", [p for p in start if s[p - 1] in "\n_" or True][0])
name_start = s.rfind("\n", 0, i) + 1
j = s.index(".Lfunc_end", i)
blocks, cur, label = [], Counter(), "entry"
for ln in s[name_start:j].split("\n"):
    t = ln.strip()
    if not t or t.startswith((";", ".section", ".p2align", ".type", ".globl")):
        continue
    if t.endswith(":"):
        blocks.append((label, cur))
        label, cur = t[:-1], Counter()
        continue
    if t.startswith("."):
        continue
    op = t.split()[0]
    k = ("mfma" if op.startswith("v_mfma") else "exp" if op.startswith("v_exp") else "cvt" if op.startswith("v_cvt")
         else "ds_read" if op.startswith("ds_read") else "ds_write" if op.startswith("ds_write")
         else "wait" if op.startswith("s_waitcnt") else "barrier" if op.startswith("s_barrier")
         else "gload" if op.startswith(("global_load", "buffer_load")) else "gstore" if op.startswith(("global_store", "global_atomic"))
         else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "other")
    cur[k] += 1
    cur["n"] += 1
blocks.append((label, cur))
for label, c in blocks:
    if c["n"] >= 8:
        print(f"{label:28s} " + " ".join(f"{k}={c[k]}" for k in ("n", "mfma", "valu", "exp", "cvt", "ds_read", "ds_write", "wait", "barrier", "gload", "gstore", "salu") if c[k]))
