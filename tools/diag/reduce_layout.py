"""Lane-level simulation of the DPP reductions: hlgs_math.h row_reduce10 (the round-5 blend backward: ten values summed
over each 16-lane row; row_reduce10_index is read off this), and the round-4 wave reduce-scatters (wave_reduce10_rs,
wave_reduce20_rs, now in tools/variants/raster_bwd_r04.hip's header era): DPP row_ror / quad_perm adds with bank masks
and the gfx950 permlane32 / permlane16 swaps, on random per-lane values; prints which value's total every lane holds.

    python tools/diag/reduce_layout.py
"""
import numpy as np
rng=np.random.default_rng(0)
def row_ror(a, n):
    out=a.copy()
    for l in range(64):
        r=l//16*16; out[l]=a[r+((l%16)-n)%16]
    return out
def dpp_add(d, a, n, bank_mask):
    src=row_ror(a,n); d=d.copy()
    for l in range(64):
        if (bank_mask>>((l%16)//4))&1: d[l]=src[l]+a[l]
    return d
def quad(a, perm):
    out=a.copy()
    for l in range(64): out[l]=a[(l&~3)+perm[l&3]]+a[l]
    return out
def p32(d,s):
    d=d.copy(); s=s.copy(); t=d[32:].copy(); d[32:]=s[:32]; s[:32]=t; return d,s
def p16(d,s):
    d=d.copy(); s=s.copy()
    for r in (0,2):
        t=d[(r+1)*16:(r+2)*16].copy(); d[(r+1)*16:(r+2)*16]=s[r*16:(r+1)*16]; s[r*16:(r+1)*16]=t
    return d,s
def fold8(a,b):
    d=np.zeros(64); d=dpp_add(d,a,8,0x3); d=dpp_add(d,b,8,0xc); return d
def fold4(a,b):
    d=np.zeros(64); d=dpp_add(d,a,12,0x5); d=dpp_add(d,b,4,0xa); return d
def check(regs, X, names):
    tot=X.sum(0)
    res={}
    for ri,r in enumerate(regs):
        for l in range(64):
            hit=[v for v in range(X.shape[1]) if abs(r[l]-tot[v])<1e-9]
            res[(ri,l)]=hit[0] if hit else None
    return res
# 10-value reference
V=10; X=rng.normal(size=(64,V))
v=[X[:,i] for i in range(V)]
s=[fold8(v[2*i],v[2*i+1]) for i in range(5)]
t1=fold4(s[2],s[3]); t0=fold4(s[0],s[1]); t2=fold4(s[4],s[4])
a,b=p32(t0,t1); t0=a+b
z=np.zeros(64); a,b=p32(t2,z); t2=a+b
a,b=p16(t0,t2); w=a+b
w=quad(w,[1,0,3,2]); w=quad(w,[2,3,0,1])
r=check([w],X,None)
print("10:", [r[(0,l)] for l in range(0,64,4)])
# 20 values
V=20; X=rng.normal(size=(64,V))
v=[X[:,i] for i in range(V)]
s=[fold8(v[2*i],v[2*i+1]) for i in range(10)]
t=[fold4(s[2*i],s[2*i+1]) for i in range(5)]
a,b=p32(t[0],t[1]); u0=a+b
a,b=p32(t[2],t[3]); u1=a+b
z=np.zeros(64); a,b=p32(t[4],z); u2=a+b
a,b=p16(u0,u1); w0=a+b
a,b=p16(u2,z); w1=a+b
for q in ([1,0,3,2],[2,3,0,1]): w0=quad(w0,q); w1=quad(w1,q)
r=check([w0,w1],X,None)
print("20 w0:", [r[(0,l)] for l in range(0,64,4)])
print("20 w1:", [r[(1,l)] for l in range(0,64,4)])
print("all lanes of a bank agree:", all(r[(ri,l)]==r[(ri,l&~3)] for ri in (0,1) for l in range(64)))

# row_reduce10: per 16-lane row
V=10; X=rng.normal(size=(64,V))
v=[X[:,i] for i in range(V)]
s=[fold8(v[2*i],v[2*i+1]) for i in range(5)]
t=[fold4(s[0],s[1]), fold4(s[2],s[3]), fold4(s[4],s[4])]
for q in ([1,0,3,2],[2,3,0,1]): t=[quad(x,q) for x in t]
ok=True
for l in range(64):
    row=l//16; tot=X[row*16:(row+1)*16].sum(0)
    beta=(l>>2)&3
    exp=[[0,2,1,3][beta],[4,6,5,7][beta],[8,8,9,9][beta]]
    for ti in range(3):
        ok &= abs(t[ti][l]-tot[exp[ti]])<1e-9
print("row_reduce10 layout as row_reduce10_index says:", ok)
