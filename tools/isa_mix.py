"""Static instruction mix of the kernels in a gfx950 assembly file (profiling
aid): python tools/isa_mix.py file.s [name-substring]."""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*;[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if want not in name:
        continue
    c = Counter()
    for line in body.split("\n"):
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        key = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else
               "waitcnt" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else
               "ds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_")) else op)
        c[key] += 1
        if op.startswith("v_div_"):
            c["(v_div_*)"] += 1
    print(name[:70], dict(c))
