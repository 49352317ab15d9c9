import sys, re
def fns(path):
    s = open(path).read()
    out = {}
    for m in re.finditer(r'^(_Z\w+):', s, re.M):
        name = m.group(1)
        end = s.find('.Lfunc_end', m.end())
        body = s[m.end():end]
        body = re.sub(r'\.LBB\d+_\d+', 'L', body)
        body = '\n'.join(l for l in body.split('\n') if not l.strip().startswith(';') and '.loc' not in l)
        out[name] = body
    return out
a, b = fns(sys.argv[1]), fns(sys.argv[2])
for k in sorted(a):
    if 'group' in k: continue
    print(('SAME ' if a[k] == b.get(k) else 'DIFF ') + k[:60], len(a[k].split('\n')), len(b.get(k, '').split('\n')))
