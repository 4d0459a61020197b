"""Access patterns of the fp16 Impala conv stack (csrc/fdr_impala_h.hip) for the bank model in check.py."""
import sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from check import *
class Lay:
    def __init__(s, CS16, CS32, fT16, fT32, fX16, fX32):
        s.CS={16:CS16,32:CS32}; s.fT={16:fT16,32:fT32}; s.fX={16:fX16,32:fX32}
    def T(s,C,q,chunk,half=0): return (q*s.CS[C] + 8*(chunk ^ s.fT[C](q)) + 4*half)//2
    def X(s,C,m,chunk,half=0): return (m*C + 8*(chunk ^ s.fX[C](m)) + 4*half)//2
def conv_reads(L,C,H,rows=None):
    W=H; WP=H+2; MT=(rows or H)*W//16; worst=1
    for mt in range(MT):
        for s in range(4 if C==16 else 9):
            a=[None]*64
            for l in range(64):
                p=l&15; g=l>>4; m=mt*16+p; q0=(m//W)*WP+m%W
                if C==16: tap=2*s+(g>>1); c=g&1
                else: tap=s; c=g
                q=q0+(tap//3)*WP+tap%3
                a[l]=L.T(C,q,c)
            worst=max(worst,degree(a,R128,4,64))
        if C==16:  # rem
            a=[None]*64
            for l in range(64):
                p=l&15; g=l>>4; m=mt*16+p; q=(m//W)*WP+m%W+2*WP+2
                a[l]=L.T(C,q,g>>1,g&1)
            worst=max(worst,degree(a,R64,2,64))
    return worst
def epi_stores(L,C,H):
    W=H; WP=H+2; worst=1
    for mt in range(H*W//16):
        for nt in range(C//16):
            a=[None]*64
            for l in range(64):
                p=l&15; g=l>>4; m=mt*16+p; q=(m//H+1)*WP+m%H+1
                a[l]=L.T(C,q,2*nt+(g>>1),g&1)
            worst=max(worst,degree(a,W64,2,32))
    return worst
def x_rmw(L,C,H):
    wr=rd=1
    for mt in range(H*H//16):
        for nt in range(C//16):
            a=[None]*64
            for l in range(64):
                p=l&15; g=l>>4; m=mt*16+p
                a[l]=L.X(C,m,2*nt+(g>>1),g&1)
            rd=max(rd,degree(a,R64,2,64)); wr=max(wr,degree(a,W64,2,32))
    return rd,wr
def to_padded(L,C,H):
    G=C//8; WP=H+2; rd=wr=1
    for w in range(0, H*H*G//64):
        a=[None]*64; b=[None]*64
        for l in range(64):
            t=64*w+l; cg=t%G; pix=t//G; y=pix//H; x=pix%H
            a[l]=L.X(C,pix,cg); b[l]=L.T(C,(y+1)*WP+x+1,cg)
        rd=max(rd,degree(a,R128,4,64)); wr=max(wr,degree(b,W128,4,32))
    return rd,wr
def report(L,name):
    out=[name]
    for C,H in ((16,32),(32,16),(32,8)):
        out.append("C%d H%d: B-read %d, epi-store %d, X rmw r/w %s, to_padded r/w %s"%(C,H,conv_reads(L,C,H),epi_stores(L,C,H),x_rmw(L,C,H),to_padded(L,C,H)))
    print("\n  ".join(out))
z=lambda q:0
if __name__=="__main__":
    report(Lay(24,40,z,z,z,z),"current")
    report(Lay(16,40,z,z,z,z),"CS16=16 (this commit)")
