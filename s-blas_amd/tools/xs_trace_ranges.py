import sys, numpy as np
L=[]
for line in open(sys.argv[1]):
    if line.startswith('#'): L.append([]); continue
    L[-1].append([int(v) for v in line.split()])
a=np.array(L[-1]); it=a[a[:,0]!=-2]
subs=[];durs=[]
for sc,ec in ((0,4),(1,5)):
    ok=it[:,sc]>=0
    subs+=list(it[ok,sc]); durs+=list((it[ok,ec]-it[ok,3])*1e-2)
subs=np.array(subs); durs=np.array(durs); rng=subs>>8
o=np.argsort(rng)
for q in np.array_split(o,8):
    w=(subs[q]&255)!=0
    print(f"ranges {rng[q].min():4d}-{rng[q].max():4d} wide {w.mean():.2f}: dur med {np.median(durs[q]):6.1f} min {durs[q].min():6.1f} max {durs[q].max():6.1f}")
