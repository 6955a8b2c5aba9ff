"""Scratch (spill) traffic and instruction counts inside a kernel's step loop
(the loop holding the DPP wave shifts) in hipcc's gfx950 assembly.
Usage: python scripts/isa_loop.py FILE.s KERNEL_SYMBOL"""
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
k = s[i:j].split('\n')
lab = 'entry'
first = next(n for n, l in enumerate(k) if 'wave_shr:1' in l)
# the loop: from the outer-loop header before the first shift to its latch
hdr = max(n for n in range(first) if 'Loop Header' in k[n] and 'Depth=1' in k[n])
hname = re.search(r'(\.LBB\d+_\d+)', k[hdr]).group(1)
latch = max(n for n, l in enumerate(k) if hname in l and 's_cbranch' in l or ('in Loop: Header=' + hname[1:].replace('LBB', 'BB')) in l)
spills = [l.strip() for l in k[hdr:latch] if 'scratch_' in l]
valu = sum(1 for l in k[hdr:latch] if re.match(r'\s+v_', l))
print(f"loop {hname}: lines {hdr}-{latch}, VALU instructions (static) {valu}, scratch ops {len(spills)}")
for x in spills:
    print("  ", x)
