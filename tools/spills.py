"""List the scratch spills / reloads of one kernel in a device-only .s file (diagnostic).
    python tools/spills.py /tmp/k.s <mangled-name-substring> [context]"""
import sys
s = open(sys.argv[1]).read()
key = sys.argv[2]
ctx = int(sys.argv[3]) if len(sys.argv) > 3 else 2
names = [l.split(';')[0].strip()[:-1] for l in s.splitlines() if l.split(";")[0].strip().endswith(":") and key in l and not l.startswith(".")]
name = names[0]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].splitlines()
print(name, len(body), 'lines')
for k, l in enumerate(body):
    if 'scratch_' in l:
        print('-----')
        for q in range(max(0, k - ctx), min(len(body), k + ctx + 1)):
            print(q, body[q])
