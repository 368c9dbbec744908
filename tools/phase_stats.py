"""Per-phase instruction / spill counts of a kernel compiled with '; PHASE <name>' asm
markers.  usage: python tools/phase_stats.py file.s kernel_regex"""
import re
import sys

L = open(sys.argv[1]).read().split('\n')
for st, l in enumerate(L):
    if not re.match(r'^_Z\S*' + sys.argv[2] + r'\S*:', l):
        continue
    en = st
    while not L[en].startswith('.Lfunc_end'):
        en += 1
    print(l.split(':')[0])
    cur, stats = 'pre', {}
    for x in L[st:en]:
        m = re.search(r'; PHASE (\S+)', x)
        if m:
            cur = m.group(1)
            continue
        d = stats.setdefault(cur, dict(n=0, scr_st=0, scr_ld=0, gld=0, div=0, bperm=0))
        if re.match(r'\s+[vsdgb]\w*_', x):
            d['n'] += 1
        d['scr_st'] += 'scratch_store' in x
        d['scr_ld'] += 'scratch_load' in x
        d['gld'] += 'global_load' in x
        d['div'] += 'v_div_fixup' in x
        d['bperm'] += 'ds_bpermute' in x
    for k, v in stats.items():
        print('  %-5s %s' % (k, v))
