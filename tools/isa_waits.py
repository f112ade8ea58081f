#!/usr/bin/env python3
"""List the s_waitcnt vmcnt sites (with line offsets and the loop header
position) of every kernel whose name matches a pattern in a hipcc .s file:
    python tools/isa_waits.py twemproxy_amd/csrc/build/kmode_6.s nc_hash_kernel_gs"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
for m in re.finditer(r'^(\S*' + pat + r'\S*):', s, re.M):
    name = m.group(1)
    start = m.end()
    end = s.find('.Lfunc_end', start)
    body = s[start:end]
    lh = body.find('Loop Header')
    vm = [(body[:w.start()].count('\n'), w.group(1)) for w in re.finditer(r's_waitcnt\s+([^\n]*vmcnt\(\d+\)[^\n]*)', body)]
    print(name, 'lines', body.count('\n'), 'loop@', body[:lh].count('\n') if lh >= 0 else None)
    for ln, w in vm:
        print('   ', ln, w)
