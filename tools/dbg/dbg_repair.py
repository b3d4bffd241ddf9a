import sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo/oracle')
import torch
import openr_amd
P = openr_amd.decision
import _refcpu as O
kind, src = "wan", "3"
opts = dict(nodes=250, seed=0xD4, prefixesPerNode=2, nodeOverloadPermille=60,
            adjOverloadPermille=60, drainPermille=80, anycastPermille=150)
n = 96
base, variants, links = O.variant_route_updates(kind, opts, src, n, 0xBEE, 700, True, True)
res = {}
for mode in (0, 1):
    vr = P.VariantRunner(True, True)
    vr.setup(kind, opts, src, n, 0xBEE, 700)
    vr.set_mode(mode)
    vr.launch(0, True)
    vr.download()
    res[mode] = [vr.canonical(v) for v in range(n)]
bad = [v for v in range(n) if res[1][v] != res[0][v]]
print("variants where repair != full:", bad)
okf = [v for v in range(n) if res[0][v] != variants[v][0]]
print("variants where full != oracle:", okf)
for v in bad[:3]:
    a, b = res[0][v].decode().splitlines(), res[1][v].decode().splitlines()
    print(v, links[v], [(x, y) for x, y in zip(a, b) if x != y][:6], len(a), len(b))
for mode in (0, 1, 2):
    vr = P.VariantRunner(True, True)
    vr.setup(kind, opts, src, n, 0xBEE, 700)
    vr.set_mode(mode)
    vr.launch(0, True)
    vr.download()
    ch = [(vr.changed(v), vr.counts(v)) for v in range(n)]
    badc = [v for v in range(n) if sorted(ch[v][0]) != variants[v][1] or ch[v][1] != (variants[v][2], variants[v][3])]
    vr.fetch_updates(0)
    badu = []
    for v in range(n):
        upd, dele = vr.update(v)
        if sorted(upd + dele) != variants[v][1]:
            badu.append(v)
    print("mode", mode, "bitmap/count mismatches", badc[:10], "update mismatches", badu[:10])
    for v in badu[:2]:
        upd, dele = vr.update(v)
        got = set(upd + dele); want = set(variants[v][1])
        print("  v", v, "extra", sorted(got - want)[:5], "missing", sorted(want - got)[:5],
              "counts", ch[v][1], (variants[v][2], variants[v][3]), "bitmap n", len(ch[v][0]))
