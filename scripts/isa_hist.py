#!/usr/bin/env python3
"""Opcode histogram of one kernel in a hipcc -S listing.  usage: isa_hist.py file.s <symbol-substring> [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
for m in re.finditer(r"^(_Z\S*):", s, re.M):
    if sys.argv[2] not in m.group(1):
        continue
    a = m.end()
    b = s.index(".Lfunc_end", a)
    ops = collections.Counter(re.findall(r"^\s+([vsd]s?_\w+|global_\w+|buffer_\w+|flat_\w+)", s[a:b], re.M))
    cls = collections.Counter()
    for k, v in ops.items():
        cls[k.split("_")[0]] += v
    print(m.group(1), sum(ops.values()), dict(cls))
    for k, v in ops.most_common(top):
        print(f"  {k:28s}{v}")
