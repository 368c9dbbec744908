"""Instruction mix of the backward-branch loops of selected kernels in a device .s file.
   usage: python tools/loop_stats.py file.s kernel_regex"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
pat = re.compile(r"^(_Z\S*" + sys.argv[2] + r"\S*):(?:\s.*)?$")
for s, l in enumerate(lines):
    m = pat.match(l)
    if not m:
        continue
    e = s
    while not lines[e].startswith('.Lfunc_end'):
        e += 1
    body = lines[s:e]
    labels = {}
    for i, x in enumerate(body):
        lm = re.match(r'^(\.LBB\S+):', x)
        if lm:
            labels[lm.group(1)] = i
    print(m.group(1), 'lines', len(body))
    for i, x in enumerate(body):
        b = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\S+)', x)
        if not b or b.group(1) not in labels or labels[b.group(1)] >= i:
            continue
        seg = body[labels[b.group(1)]:i]

        def cnt(p):
            return sum(1 for y in seg if re.match(r'\s+' + p, y))
        f64 = sum(1 for y in seg if re.search(r'v_\w+_f64', y))
        dpp = sum(1 for y in seg if re.search(r'(row_|wave_|dpp)', y))
        print('  loop %s span %d: v_=%d f64=%d dpp=%d vmem_ld=%d vmem_st=%d s_=%d waitcnt=%d' % (
            b.group(1), i - labels[b.group(1)], cnt('v_'), f64, dpp, cnt('(?:global|buffer)_load'),
            cnt('(?:global|buffer)_store'), cnt('s_'), cnt('s_waitcnt')))
