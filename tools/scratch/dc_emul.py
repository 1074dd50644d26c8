# Numpy emulation of dc_block_kernel / dc_carry_kernel (misc_kernels.hip) against the oracle's serial
# DC removal + pre-emphasis: the round-4 lane-dense scan's rounding (DESIGN.md Kernel 4).  CPU only.
import numpy as np, sys
sys.path.insert(0,'oracle')
import oracle as O
rng=np.random.default_rng(1)
n=300_000
x=rng.standard_normal(n)+0.3
R=0.995; alpha=0.95
ref=O.preemphasis(O.dc_removal(x,R),alpha)
L=8; BLK=256*L
def pw(r,k):
    v=1.0
    for _ in range(k): v*=r
    return v
R16=pw(R,L); RC=pw(R,BLK)
T=(n+BLK-1)//BLK
xp=np.concatenate([[0.0],x])
def chunk_e(b):
    base=b*BLK
    e=np.zeros(256)
    for c in range(256):
        s=base+L*c; y=0.0
        for j in range(L):
            if s+j<n: y=(xp[s+j+1]-xp[s+j])+R*y
        e[c]=y
    return e
def scan(e):
    # kogge-stone per wave then waves composite
    B=e.copy(); A=np.full(256,R16)
    for w in range(4):
        Bw=B[64*w:64*w+64]; Aw=A[64*w:64*w+64]
        d=1
        while d<64:
            Bp=np.concatenate([np.zeros(d),Bw[:-d]]); Ap=np.concatenate([np.ones(d),Aw[:-d]])
            m=np.arange(64)>=d
            Bn=np.where(m,Bw+Aw*Bp,Bw); An=np.where(m,Aw*Ap,Aw)
            Bw,Aw=Bn,An; d*=2
        B[64*w:64*w+64]=Bw; A[64*w:64*w+64]=Aw
    comp=[]
    Bc,Ac=0.0,1.0
    for w in range(4):
        comp.append((Bc,Ac))
        Bc=B[64*w+63]+A[64*w+63]*Bc; Ac=A[64*w+63]*Ac
    return B,A,comp
ends=np.zeros(T)
for b in range(T):
    B,A,comp=scan(chunk_e(b)); Bw,Aw=comp[3]
    ends[b]=B[255]+A[255]*Bw
ys=np.zeros(T); Y=0.0
for b in range(T):   # serial carry (scan differs by ulps; fine for the estimate)
    ys[b]=Y; Y=ends[b]+RC*Y
z=np.zeros(n)
for b in range(T):
    B,A,comp=scan(chunk_e(b)); base=b*BLK; Yb=ys[b]
    for c in range(256):
        w=c//64; Bw,Aw=comp[w]
        if c%64==0: Be,Ae=0.0,1.0
        else: Be,Ae=B[c-1],A[c-1]
        Be=Be+Ae*Bw; Ae=Ae*Aw
        y1=Yb if c==0 else Be+Ae*Yb
        s=base+L*c
        for j in range(L):
            if s+j>=n: break
            yv=(xp[s+j+1]-xp[s+j])+R*y1
            z[s+j]=yv-alpha*y1; y1=yv
err=np.abs(z-ref)
print("max abs err", err.max(), "rel to max|ref|", err.max()/np.abs(ref).max(), "max |ref|", np.abs(ref).max())
e1=O.short_time_energy(ref,1024,256); e2=O.short_time_energy(z,1024,256)
print("energy rel", np.max(np.abs(e1-e2)/e1))
