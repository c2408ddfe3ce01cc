"""Static gfx950 instruction mix per kernel from a `hipcc --cuda-device-only -S` listing."""
import collections, re, sys
src = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2:] or ['']
cur, body = None, []
out = {}
for l in src:
    m = re.match(r'^(_Z[\w]+):', l)
    if m:
        cur, body = m.group(1), []
        continue
    if cur and l.startswith('.Lfunc_end'):
        out[cur] = body
        cur = None
        continue
    if cur:
        t = l.strip()
        if t and not t.startswith(('.', ';', '//')) and not re.match(r'^[\w.$]+:', t):
            body.append(t.split()[0])
for name, ins in out.items():
    if not any(p in name for p in pat):
        continue
    c = collections.Counter(i.split('_')[0] for i in ins)
    f64 = sum(1 for i in ins if i.endswith('_f64'))
    print(f"{name[:70]:70s} total {len(ins):5d} v {c['v']:5d} (f64 {f64}) s {c['s']:4d} ds {c['ds']:3d} "
          f"global {c['global'] + c['buffer'] + c['flat']:3d}")
