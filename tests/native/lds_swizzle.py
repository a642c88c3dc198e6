"""LDS bank-conflict model of k_ntt8's layouts (TUNING ONLY; not collected by pytest).

Replays every LDS access of a 10-stage pass in 512-thread blocks (rows of 4 felts):
the compute rounds of both directions (coord_q / coord_gg of csrc/ntt.hip) and the
staged column walks, and counts conflicts with the banking of MI355X_MICROARCH.md
SS LDS: ds_read_b128 in four 16-lane groups over a 256-B line, ds_write_b128 in
eight 8-lane groups over a 128-B line. `lidx_new` is the layout in csrc/ntt.hip;
`lidx_par` the first (row-parity) attempt, whose read conflicts rocprofv3 measured
(SQ_LDS_BANK_CONFLICT 6.4e8 -> 0 with lidx_new).
"""
import itertools
K=10; LOGNT=9; logT=LOGNT+3-K; T=1<<logT
def rounds(K):
    n=(K+2)//3; rem=K; out=[]
    for r in range(n):
        left=n-r; b=(rem+left-1)//left; b=min(b,3); out.append(b); rem-=b
    return out
def bit(q,i): return (q>>i)&1
def lidx_new(q,x):
    h0=bit(q,2)^bit(q,3); h1=bit(q,2)^bit(q,5)
    P=q^(h0|(h1<<1))
    s=bit(q,1)|((bit(q,2)^bit(q,3))<<1)
    return P*T+(x^s)
def lidx_par(q,x):
    return ((q&~1)|(bin(q).count('1')&1))*T+(x^((q>>1)&3))
RG=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
RG+= [[l+32 for l in g] for g in RG]
def conflicts(addrs, write):
    c=0
    groups=[list(range(i,i+8)) for i in range(0,64,8)] if write else RG
    for g in groups:
        slots={}
        for l in g:
            a=addrs[l]; s=a%8 if write else a%16
            slots.setdefault(s,set()).add(a)
        c+=sum(len(v)-1 for v in slots.values())
    return c
def check(lidx):
    tot={'cr':0,'cw':0,'sr':0,'sw':0}
    for dit in (True,False):
        rbs=rounds(K); b0=0 if dit else K
        for rb in rbs:
            if not dit: b0-=rb
            for wave in range(8):
                for m in range(8):
                    addrs=[]
                    for lane in range(64):
                        tid=wave*64+lane
                        extra=m>>rb; bf=m&((1<<rb)-1)
                        c=(extra<<LOGNT)|tid
                        gg=c&(T-1); qo=c>>logT
                        ql=qo&((1<<b0)-1)
                        q=((qo>>b0)<<(b0+rb))|(bf<<b0)|ql
                        addrs.append(lidx(q,gg))
                    tot['cr']+=conflicts(addrs,False); tot['cw']+=conflicts(addrs,True)
            if dit: b0+=rb
    # staged: Tl=1 (column walk) and Tl=T
    for Tl in (1,T):
        logTl=Tl.bit_length()-1
        for wave in range(8):
            for i in range(8):
                addrs=[]
                for lane in range(64):
                    e=wave*64+lane+i*512
                    ll=e&(Tl-1); rest=e>>logTl; q=rest&((1<<K)-1); hl=rest>>K
                    addrs.append(lidx(q,hl*Tl+ll))
                tot['sr']+=conflicts(addrs,False); tot['sw']+=conflicts(addrs,True)
    return tot
print('parity', check(lidx_par))
print('new   ', check(lidx_new))


def lidx_product(q, x, T):
    """conflict-free layouts per row length (rows of 4: csrc/ntt.hip's lidx; rows of
    8 and >= 32: measured no faster than the product's x ^ (q & 7))"""
    if T >= 32:
        return q * T + (x ^ (q & 15))
    if T == 16:
        return q * T + (x ^ (q & 7))
    if T == 8:
        return (q ^ (((q >> 2) ^ (q >> 3)) & 1)) * T + (x ^ (q & 7))
    h0 = ((q >> 2) ^ (q >> 3)) & 1
    h1 = ((q >> 2) ^ (q >> 5)) & 1
    return (q ^ (h0 | (h1 << 1))) * T + (x ^ (((q >> 1) & 1) | (h0 << 1)))


if __name__ == "__main__":
    import re
    base = open(__file__).read().split("RG=[")[0]
    for K, LOGNT in [(5, 8), (6, 8), (7, 8), (8, 8), (9, 9), (10, 9)]:
        g = {}
        code = open(__file__).read().split("print('parity'")[0]
        code = code.replace("K=10; LOGNT=9", f"K={K}; LOGNT={LOGNT}")
        code = code.replace("i*512", f"i*{1 << LOGNT}").replace("for wave in range(8)", f"for wave in range({(1 << LOGNT) // 64})")
        exec(code, g)
        T = g["T"]
        print(f"K={K:2d} T={T:2d}", g["check"](lambda q, x: lidx_product(q, x, T)))


def lidx_rows_of_1(q, x):
    """csrc/ntt.hip's rows of 1 felt (11-stage passes in 256-thread blocks, 2^19-2^20):
    slot bits 0-2 ^= q bits 3-5, slot bit 3 ^= q bit 6."""
    return q ^ ((q >> 3) & 7) ^ (((q >> 6) & 1) << 3)


if __name__ == "__main__":
    for K, LOGNT in [(11, 8), (9, 8)]:
        g = {}
        code = open(__file__).read().split("print('parity'")[0]
        code = code.replace("K=10; LOGNT=9", f"K={K}; LOGNT={LOGNT}")
        code = code.replace("i*512", f"i*{1 << LOGNT}").replace("for wave in range(8)", f"for wave in range({(1 << LOGNT) // 64})")
        exec(code, g)
        T = g["T"]
        lidx = (lambda q, x: lidx_rows_of_1(q, x)) if T == 1 else (lambda q, x: lidx_product(q, x, T))
        print(f"two-pass plan K={K:2d} T={T}", g["check"](lidx))



def lidx_r06(q, x, T):
    """csrc/ntt.hip's layouts from round 6 on: conflict-free for every pass shape the
    library launches (rows of 16: the DIF passes' layout, found by a search over one
    extra q-bit parity in felt bit 3; the DIT passes keep x ^ (q & 7), conflict-free in
    their rounds, because this one measured 1-3% slower there)."""
    if T == 1:
        return lidx_rows_of_1(q, x)
    if T >= 32:
        return q * T + (x ^ (q & 15))
    if T == 16:
        return q * T + (x ^ ((q & 7) | ((((q >> 2) ^ (q >> 4)) & 1) << 3)))
    if T == 8:
        return (q ^ (((q >> 2) ^ (q >> 3)) & 1)) * T + (x ^ (q & 7))
    return lidx_product(q, x, T)


if __name__ == "__main__":
    for K, LOGNT in [(5, 8), (6, 8), (7, 8), (8, 8), (9, 8), (9, 9), (11, 8)]:
        g = {}
        code = open(__file__).read().split("print('parity'")[0]
        code = code.replace("K=10; LOGNT=9", f"K={K}; LOGNT={LOGNT}")
        code = code.replace("i*512", f"i*{1 << LOGNT}").replace("for wave in range(8)", f"for wave in range({(1 << LOGNT) // 64})")
        exec(code, g)
        T = g["T"]
        r = g["check"](lambda q, x: lidx_r06(q, x, T))
        print(f"r06 K={K:2d} NT={1 << LOGNT} T={T:2d}", r)
        assert sum(r.values()) == 0
