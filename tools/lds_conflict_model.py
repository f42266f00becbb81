#!/usr/bin/env python3
"""LDS bank model of k_conv3lg<W, 1>'s in-place GroupNorm transform (csrc/conv3l.hip tdst[]): the
ds_read_b128 (4 x 16 lane groups, bank slot (a/16) mod 16) and ds_write_b128 (8 x 8 contiguous lanes,
bank slot (a/16) mod 8) cycles of one unit access per (row width, wave parity, group, unit index),
from the lane groups of MI355X_MICROARCH.md's LDS table.  Ideal: 4 read and 8 write cycles.
usage: python tools/lds_conflict_model.py"""
import itertools, random
RG=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
RG=RG+[[x+32 for x in g] for g in RG]
WG=[list(range(8*k,8*k+8)) for k in range(8)]
def sw(col): return (col>>2)&3
def setup(W, wvodd, tg, i):
    W2=W+2; L_TP=256; NPX=(L_TP//W+2)*W2
    res=[]
    for lane in range(64):
        hp0=wvodd*64+lane+128*i
        hp=hp0 if hp0<NPX else NPX+(lane&3)
        hc=hp%W2
        res.append(hp*64+16*((2*tg)^sw(hc)))
    return res
def rdeg(addrs):
    tot=0
    for g in RG:
        from collections import defaultdict
        d=defaultdict(set)
        for l in g: d[(addrs[l]//16)%16].add(addrs[l])
        tot+=max(len(v) for v in d.values())
    return tot  # sum of per-group cycles (ideal 4)
def wdeg(addrs):
    tot=0
    for g in WG:
        from collections import defaultdict
        d=defaultdict(set)
        for l in g: d[(addrs[l]//16)%8].add(addrs[l])
        tot+=max(len(v) for v in d.values())
    return tot  # ideal 8
for W in (32,64):
    TU=4 if W==64 else 3
    for wvodd in (0,1):
        for tg in (0,1):
            for i in range(TU):
                a=setup(W,wvodd,tg,i); b=[x^16 for x in a]
                print(W,wvodd,tg,i,"read",rdeg(a),rdeg(b),"write",wdeg(a),wdeg(b))
