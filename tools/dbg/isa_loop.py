"""Print the vector-memory loads and vmcnt waits of one kernel in a hipcc -S listing, with loop
labels, to check how many gathers stay in flight:
    python tools/dbg/isa_loop.py <file.s> <mangled-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
name = [m.group(1) for m in re.finditer(r'^(\S+):', s, re.M) if sys.argv[2] in m.group(1)][0]
i = s.index(name + ':')
body = s[i:s.index('.Lfunc_end', i)].split('\n')
print(name)
for k, l in enumerate(body):
    if re.search(r'global_load|vmcnt|Loop Header|^\.LBB|s_cbranch|s_branch', l):
        print(k, l.strip()[:90])
