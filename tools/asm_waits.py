#!/usr/bin/env python3
"""Per-kernel count of global loads vs `s_waitcnt vmcnt(0)` in a hipcc -save-temps .s file
(a high vmcnt(0)-per-load ratio flags serialised loads)."""
import re
import sys

for path in sys.argv[1:]:
    s = open(path).read()
    for m in re.finditer(r'^(_Z\S+):\s*;', s, re.M):
        name = m.group(1)
        j = s.find('s_endpgm', m.end())
        body = s[m.end():j]
        nl = len(re.findall(r'global_load_(?!lds)', body))
        nw = len(re.findall(r's_waitcnt vmcnt\(0\)', body))
        print(f"{name[:90]:92s} loads={nl:4d} vmcnt0={nw:4d}")
