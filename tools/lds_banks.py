"""LDS bank-conflict model (MI355X_MICROARCH.md §LDS lane groups / bank rules) for the 256x256
GEMM fragment reads: the K-contiguous (ds_read_b128) and MN-contiguous (ds_read_b64_tr_b16) B
images under the interleaved column order of the swapped-operand kernel, and a search over XOR
swizzles. python tools/lds_banks.py"""
# LDS bank-conflict model for the G8 fragment reads (MI355X_MICROARCH.md §LDS)
import itertools
G128=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128+= [[x+32 for x in g] for g in G128]
def cyc128(addrs):
    tot=0
    for grp in G128:
        banks={}
        for l in grp:
            a=addrs[l]
            for d in range(4):
                b=(a//4+d)%64
                banks.setdefault(b,set()).add(a//16)
        tot+=max(len(v) for v in banks.values())
    return tot
def cyc64(addrs):
    tot=0
    for h in (range(0,32),range(32,64)):
        banks={}
        for l in h:
            a=addrs[l]
            for d in range(2):
                b=(a//4+d)%64
                banks.setdefault(b,set()).add(a//8)
        tot+=max(len(v) for v in banks.values())
    return tot
def col_remap(j,i): return 8*(i>>2)+4*j+(i&3)
# layout 0: rows of 128B, swz(r,c)=c^h(r)
def l0_cycles(h, remap):
    worst=0
    for wc in range(4):
      for j in range(2):
        for kc in range(2):
            addrs=[]
            for l in range(64):
                g,i=l>>4,l&15
                row = wc*32 + (col_remap(j,i) if remap else j*16+i)
                addrs.append(row*128 + ((kc*4+g) ^ h(row))*16)
            worst=max(worst,cyc128(addrs))
    return worst
print("l0 existing swizzle, no remap:", l0_cycles(lambda r: r&7, False))
print("l0 existing swizzle, remap:", l0_cycles(lambda r: r&7, True))
best=None
for M in itertools.product(range(8), repeat=4):  # h(r) = xor of M[b] for bits b of r&15
    h=lambda r,M=M: (M[0] if r&1 else 0)^(M[1] if r&2 else 0)^(M[2] if r&4 else 0)^(M[3] if r&8 else 0)
    c=l0_cycles(h,True)
    if best is None or c<best[0]: best=(c,M)
    if c==4: break
print("best l0 remap:", best)
# layout 1: [64 k-rows][256B], 8B units; swz on 16B chunk
def l1_cycles(h, remap):
    worst=0
    for wc in range(4):
      for j in range(2):
        for kc in range(2):
          for second in range(2):
            addrs=[]
            for l in range(64):
                g,i=l>>4,l&15
                q,p=i>>2,i&3
                r=kc*32+8*g+q+4*second
                u = wc*8 + (2*p+j if remap else j*4+p)
                addrs.append(r*256 + ((u>>1) ^ h(r))*16 + (u&1)*8)
            worst=max(worst,cyc64(addrs))
    return worst
h1=lambda r: 2*((r&3)|(((r>>3)&1)<<2))
print("l1 existing, no remap:", l1_cycles(h1,False), " remap:", l1_cycles(h1,True))
best=None
for M in itertools.product(range(16), repeat=4):
    h=lambda r,M=M: (M[0] if r&1 else 0)^(M[1] if r&2 else 0)^(M[2] if r&4 else 0)^(M[3] if r&8 else 0)
    c=l1_cycles(h,True)
    if best is None or c<best[0]: best=(c,M)
    if c==2: break
print("best l1 remap:", best)
print("---- sigma map")
SIG=[0,2,1,3]
def U(j,p): return 2*SIG[p] + ((p&1) if j==0 else 1-(p&1))
col_remap = lambda j,i: 4*U(j,i>>2)+(i&3)
def l1_cycles2(h):
    worst=0
    for wc in range(4):
      for j in range(2):
        for kc in range(2):
          for second in range(2):
            addrs=[]
            for l in range(64):
                g,i=l>>4,l&15
                q,p=i>>2,i&3
                r=kc*32+8*g+q+4*second
                u = wc*8 + U(j,p)
                addrs.append(r*256 + ((u>>1) ^ h(r))*16 + (u&1)*8)
            worst=max(worst,cyc64(addrs))
    return worst
print("l1 sigma map existing swizzle:", l1_cycles2(h1))
print("l0 sigma map existing swizzle:", l0_cycles(lambda r: r&7, True))
best=None
for M in itertools.product(range(8), repeat=4):
    h=lambda r,M=M: (M[0] if r&1 else 0)^(M[1] if r&2 else 0)^(M[2] if r&4 else 0)^(M[3] if r&8 else 0)
    c=l0_cycles(h,True)
    if best is None or c<best[0]: best=(c,M)
    if c==4: break
print("best l0 sigma:", best)
print("---- same-parity maps")
for SG in itertools.permutations(range(4)):
    Uf=lambda j,p,SG=SG: 2*SG[p]+j
    col_remap = lambda j,i,Uf=Uf: 4*Uf(j,i>>2)+(i&3)
    U = Uf
    print(SG, "l0:", l0_cycles(lambda r: r&7, True), "l1:", l1_cycles2(h1))
