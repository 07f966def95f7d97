"""Print the memory loads, waits, branches and labels of one kernel in a hipcc -S listing:
    python tools/dbg/isa_loads.py <file.s> <mangled-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r'^(\S+):\s*(?:;.*)?$', s, re.M) if sys.argv[2] in m.group(1)
         and not m.group(1).startswith('.')]
name = names[0]
i = s.index(name + ':')
body = s[i:s.index('.Lfunc_end', i)].split('\n')
print(name, len(body), 'lines')
for k, l in enumerate(body):
    if re.search(r'global_load|s_waitcnt|s_cbranch|^\.LBB|buffer_load|global_store|v_readlane|s_barrier', l):
        print(k, l.strip())
