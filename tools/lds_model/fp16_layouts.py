"""Conflict degrees of every modelled fp16 conv LDS access: the chosen chunk swizzles (tsw / xsw in
fdr_impala_h.hip) vs the r05 padded, unswizzled layouts.  python tools/lds_model/fp16_layouts.py"""
from model import *  # noqa: F401,F403
t16=lambda q:(q>>3)&1; t32=lambda q:(q>>1)&3; x16=lambda m:(m>>3)&1; x32=lambda m:(m>>2)&3
L=Lay(16,32,t16,t32,x16,x32)
report(L,"chosen")
Lz=Lay(24,40,z,z,z,z)
def rem(L):
    C,H=16,32; W=H; WP=H+2; w=1
    for mt in range(64):
        a=[None]*64
        for l in range(64):
            p=l&15; g=l>>4; m=mt*16+p; q=(m//W)*WP+m%W+2*WP+2
            a[l]=L.T(C,q,g>>1,g&1)
        w=max(w,degree(a,R64,2,64))
    return w
print("rem read chosen", rem(L), "current", rem(Lz))
def breads_only(L,C,H):
    W=H; WP=H+2; worst=1
    for mt in range(H*W//16):
        for s in range(4 if C==16 else 9):
            a=[None]*64
            for l in range(64):
                p=l&15; g=l>>4; m=mt*16+p; q0=(m//W)*WP+m%W
                if C==16: tap=2*s+(g>>1); c=g&1
                else: tap=s; c=g
                q=q0+(tap//3)*WP+tap%3
                a[l]=L.T(C,q,c)
            worst=max(worst,degree(a,R128,4,64))
    return worst
for C,H in ((16,32),(32,16),(32,8)): print("full-step B reads",C,H,"chosen",breads_only(L,C,H),"current",breads_only(Lz,C,H))
# stage entry: S stores, pool reads, pool X writes
def entry(L,COUT,H,BR):
    G=COUT//8; HO=H//2; PRB=(BR-1)//2; st=pr_=pw=1
    MT=BR*H//16
    for mt in range(MT):
        for nt in range(COUT//16):
            a=[None]*64
            for l in range(64):
                p=l&15; g=l>>4; m=mt*16+p
                a[l]=L.X(COUT,m,2*nt+(g>>1),g&1)
            st=max(st,degree(a,W64,2,32))
    NI=PRB*HO*G
    for w in range((NI+63)//64):
        for dr in range(3):
            for col in range(3):
                a=[None]*64; b=[None]*64
                for l in range(64):
                    i=64*w+l
                    if i>=NI: continue
                    cg=i%G; r=i//G; px=r%HO; pr=r//HO
                    xl=2*px-1 if px>0 else 0
                    x=(xl,2*px,2*px+1)[col]
                    a[l]=L.X(COUT,(2*pr+dr)*H+x,cg)
                    b[l]=L.X(COUT,pr*HO+px,cg)
                pr_=max(pr_,degree(a,R128,4,64)); pw=max(pw,degree(b,W128,4,32))
    return st,pr_,pw
for COUT,H,BR in ((16,64,33),(32,32,17),(32,16,17)):
    print("entry",COUT,H,"chosen (S store, pool read, X write)",entry(L,COUT,H,BR),"current",entry(Lz,COUT,H,BR))
