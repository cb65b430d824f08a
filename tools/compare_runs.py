#!/usr/bin/env python3
"""Bitwise comparison of determinism.py outputs (first file vs each other one).  Diagnostic only.
    python tools/compare_runs.py a.npz b.npz ..."""
import numpy as np, sys
d={k:np.load(k) for k in sys.argv[1:]}
def cmp(a,b):
    A,B=d[a],d[b]
    tot=0
    for k in range(A['U'].shape[0]):
        du=np.abs(A['U'][k]-B['U'][k]).max(axis=0)
        nd=(du>0).sum(); fd=(A['flag'][k]!=B['flag'][k]).sum(); tot+=nd
        if nd or fd: print(f'  {a} vs {b} step {k}: U differs in {nd} scenarios, max {du.max():.3e}, flags differ {fd}; first ids {np.flatnonzero(du>0)[:5]}')
    print(a,b,'total differing', tot)
names=list(d)
for i in range(1,len(names)): cmp(names[0],names[i])
for n in d: print(n, dict(zip(*np.unique(d[n]['flag'][-1],return_counts=True))))
