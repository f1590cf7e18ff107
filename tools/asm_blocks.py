"""Instruction mix per basic block of one kernel in gr_hip.s (make -C 3dgaussian_amd/csrc asm):
python tools/asm_blocks.py <asm> <kernel-name-substring>"""
import re, sys
s = open(sys.argv[1]).read()
m = re.search(r'\n(_Z\S*' + re.escape(sys.argv[2]) + r'\S*):', s)
i = m.start() + 1
j = s.find('.Lfunc_end', i)
body = s[i:j].split('\n')
labels = [(k, l) for k, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)]
for (k, l), (k2, _) in zip(labels, labels[1:] + [(len(body), '')]):
    ins = [x.strip() for x in body[k:k2] if x.startswith('\t') and not x.strip().startswith(('.', ';'))]
    nv = sum(1 for x in ins if x.startswith('v_') and 'mfma' not in x)
    nm = sum(1 for x in ins if 'mfma' in x)
    ne = sum(1 for x in ins if x.startswith('v_exp'))
    nds = sum(1 for x in ins if x.startswith('ds_'))
    npk = sum(1 for x in ins if x.startswith('v_pk_'))
    ncvt = sum(1 for x in ins if x.startswith('v_cvt'))
    ns = sum(1 for x in ins if x.startswith('s_'))
    br = [x for x in ins if x.startswith('s_cbranch') or x.startswith('s_branch')]
    print(f"{l:14s} n={len(ins):4d} valu={nv:4d} (pk {npk}, cvt {ncvt}) mfma={nm:3d} exp={ne:3d} ds={nds:3d} salu={ns:3d} {br[-1] if br else ''}")
