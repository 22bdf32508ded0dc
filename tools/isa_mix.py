"""Instruction mix of the LDS-read-to-write segments of one kernel in a disassembly (tools/disasm.py output):
python tools/isa_mix.py <file.s> <mangled-kernel-name-substring>. One line per segment (a run of ds_read that
starts a node body, up to its last ds_write): start index, reads, VALU, SALU, frequent opcodes."""
import re
import sys

L = open(sys.argv[1]).read().splitlines()
heads = [i for i, l in enumerate(L) if re.match(r"^[0-9a-f]+ <", l)]
st = [i for i in heads if sys.argv[2] in L[i]][0]
en = min([i for i in heads if i > st] + [len(L)])
ins = [(m.group(1), l) for l in L[st:en] for m in [re.match(r"\s+([a-z_0-9]+)\s", l)] if m]
rd = ("ds_read_b128", "ds_read_b64", "ds_read_b32")
i = 0
while i < len(ins):
    if ins[i][0] in rd:
        k = i
        while k < len(ins) and not ins[k][0].startswith("ds_write"):
            k += 1
        nxt = k
        while nxt < len(ins) and ins[nxt][0] not in rd:
            nxt += 1
        last = max([q for q in range(k, nxt) if ins[q][0].startswith("ds_write")] or [k])
        seg = ins[i:last + 1]
        cnt = {}
        for n, _ in seg:
            cnt[n] = cnt.get(n, 0) + 1
        valu = sum(v for n, v in cnt.items() if n.startswith("v_"))
        salu = sum(v for n, v in cnt.items() if n.startswith("s_") and n not in ("s_waitcnt", "s_nop"))
        nr = sum(v for n, v in cnt.items() if n in rd)
        print(i, nr, valu, salu, {n: v for n, v in cnt.items() if v >= 6 and n.startswith("v_")})
        i = last + 1
    else:
        i += 1
