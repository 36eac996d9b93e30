"""Static scan of a kernel's gfx950 assembly (hipcc -save-temps): compiler-inserted vmcnt waits,
barriers and the register counts, to check that a pipelined kernel's loads stay in flight.
  python tools/asm_waits.py <file.s> <kernel-name-substring> [...]"""
import re
import sys


def scan(path, pats):
    S = open(path).read()
    s = S.splitlines()
    for k, l in enumerate(s):
        m = re.match(r'^(_Z\S+):', l)
        if not m or not any(p in m.group(1) for p in pats):
            continue
        name = m.group(1)
        j = k
        while not s[j].startswith('.Lfunc_end'):
            j += 1
        body = s[k:j]
        comp = [i for i, x in enumerate(body) if 's_waitcnt' in x and 'vmcnt' in x and 'ASMSTART' not in body[i - 1]]
        v0 = [i for i in comp if 'vmcnt(0)' in body[i]]
        md = re.search(r'\.name:\s+' + re.escape(name) + r'\n(.*?)\.vgpr_count:\s+(\d+)', S, re.S)
        spill = re.search(r'\.vgpr_spill_count:\s+(\d+)', md.group(1)) if md else None
        print(f"{name[:70]:70s} lines {len(body):5d} compiler vmcnt waits {len(comp):3d} (vmcnt(0): {len(v0)}) "
              f"barriers {sum('s_barrier' in x for x in body)} vgpr {md.group(2) if md else '?'}")


if __name__ == "__main__":
    scan(sys.argv[1], sys.argv[2:])
