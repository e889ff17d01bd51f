"""Loop / spill map of one kernel in a gfx950 .s file: python tools/asmloops.py all.s <kernel-substring>."""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
VM0 = r"vmcnt\(0\)"
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
open("/tmp/asm/kernel.s", "w").write("\n".join(body))
labels = {m.group(1): n for n, l in enumerate(body) if (m := re.match(r"^(\.LBB\S+):", l))}
print("kernel lines", len(body))
for n, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+ (\.LBB\S+)|s_branch (\.LBB\S+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if labels.get(t, 1 << 30) < n:
            seg = body[labels[t]:n]
            cnt = lambda p: sum(1 for x in seg if re.search(p, x))
            print(f"loop {labels[t]}-{n}: instr {sum(1 for x in seg if x.startswith(chr(9)) and not x.strip().startswith(';'))}"
                  f" ds_read {cnt(r'ds_read')} ds_write {cnt(r'ds_write')} buf {cnt(r'buffer_')} glob {cnt(r'global_')}"
                  f" scratch_ld {cnt(r'scratch_load')} scratch_st {cnt(r'scratch_store')} vmcnt0 {cnt(VM0)} waitcnt {cnt(r's_waitcnt')}")
