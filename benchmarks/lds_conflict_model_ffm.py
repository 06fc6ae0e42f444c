import itertools
F=39; FF=F*F; TPB=256; NS=(FF+255)//256
R128=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
R128=R128+[[x+32 for x in g] for g in R128]
W128=[list(range(8*i,8*i+8)) for i in range(8)]
def conflicts(addrs, groups, nb, width):
    extra=0
    for g in groups:
        banks={}
        for k in g:
            a=addrs[k]
            if a is None: continue
            for d in range(width):
                banks.setdefault((a+d)%nb,set()).add(a+d)
        extra+=max((len(v) for v in banks.values()),default=1)-1
    return extra
def ab(s):
    if s>=FF: return 0,0
    return s//F, s%F
def run(stride):   # stride: dwords per transposed row (F*4 = 156 default)
    tot={'tr_read':0,'tr_write':0,'rm_read':0,'sm_a':0,'sm_b':0}; n=0
    for w in range(4):
        for j in range(NS):
            lanes=[w*64+k+j*TPB for k in range(64)]
            tr=[ (ab(s)[1]*stride + ab(s)[0]*4) for s in lanes]
            rm=[ (s if s<FF else 0)*4 for s in lanes]
            sa=[ ab(s)[0]*4 for s in lanes]; sb=[ab(s)[1]*4 for s in lanes]
            tot['tr_read']+=conflicts(tr,R128,64,4); tot['tr_write']+=conflicts(tr,W128,32,4)
            tot['rm_read']+=conflicts(rm,R128,64,4); tot['sm_a']+=conflicts(sa,R128,64,4); tot['sm_b']+=conflicts(sb,R128,64,4)
            n+=1
    return {k:v/n for k,v in tot.items()}
for st in (156,160,164,172,188):
    print(st, run(st))
