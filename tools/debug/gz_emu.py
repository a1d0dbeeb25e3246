import sys, zlib, gzip, struct
sys.path.insert(0,'/root/repo')
from tests import corpus, oracle_lib
LB=[3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE=[0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DB=[1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DE=[0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
def rev(v,n): return int(format(v,'0%db'%n)[::-1],2) if n else 0
def litcode(s):
    if s<144: return rev(0x30+s,8),8
    if s<256: return rev(0x190+s-144,9),9
    if s<280: return rev(s-256,7),7
    return rev(0xC0+s-280,8),8
def block(tb, final):
    n=len(tb); ht=[0]*4096; ml=[0]*n; md=[0]*n
    for p0 in range(0,n,64):
        hs={}
        for lane in range(64):
            p=p0+lane
            if p+4>n: continue
            w=tb[p]|tb[p+1]<<8|tb[p+2]<<16|tb[p+3]<<24
            h=((w*2654435761)&0xffffffff)>>20
            prev = hs[h]+1 if h in hs else ht[h]
            hs[h]=p
            L=0
            if prev:
                j=prev-1; lim=min(n-p,258)
                while L<lim and tb[j+L]==tb[p+L]: L+=1
            ml[p]=L if L>=4 else 0; md[p]=p+1-prev if prev else 0
        for h,p in hs.items(): ht[h]=p+1
    bits=[]  # (value,nbits)
    bits.append((final|2,3))
    p=0
    while p<n:
        L=ml[p]
        if L:
            ls=max(i for i in range(29) if LB[i]<=L); d=md[p]; ds=max(i for i in range(30) if DB[i]<=d)
            c,nb=litcode(257+ls); bits+= [(c,nb),(L-LB[ls],LE[ls]),(rev(ds,5),5),(d-DB[ds],DE[ds])]
            p+=L
        else:
            bits.append(litcode(tb[p])); p+=1
    bits.append(litcode(256))
    return bits
def member(text):
    out=[]; SUB=4096
    nb = max(1,(len(text)+SUB-1)//SUB)
    for b in range(nb): out+=block(text[b*SUB:(b+1)*SUB], 1 if b==nb-1 else 0)
    acc=0; na=0; by=bytearray()
    for v,n in out:
        acc|=v<<na; na+=n
        while na>=8: by.append(acc&255); acc>>=8; na-=8
    if na: by.append(acc&255)
    return b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff"+bytes(by)+struct.pack("<II", zlib.crc32(text), len(text)&0xffffffff)
def main():
    import starch_amd
    c = starch_amd.Starch(0); c.set_compression_method(starch_amd.K_GZIP)
    for name, d in (("cfg1", corpus.cfg1_bed(10000)), ("multi", corpus.multi_chrom_bed(5, 3000, seed=4, kind="bed6")),
                    ("fuzz", corpus.parseable_fuzz_bed(7, 4000)), ("fuzz2", corpus.parseable_fuzz_bed(7, 4000))):
        idx, members = starch_amd.parse_archive(c.compress(d))
        _, segs = oracle_lib.transform(d)
        print(name, len(segs), len(members))
        for k, ((ch, n, t), g) in enumerate(zip(segs, members)):
            e = member(t)
            if e != g:
                i = next((i for i in range(min(len(e), len(g))) if e[i] != g[i]), min(len(e), len(g)))
                print(" seg", k, ch, "len", len(t), "emu", len(e), "gpu", len(g), "first diff byte", i, "bit", (i - 10) * 8,
                      "emu", e[i:i+8].hex(), "gpu", g[i:i+8].hex())
    print("done")
main()
