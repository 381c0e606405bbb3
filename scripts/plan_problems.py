import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json, sys, numpy as np
from collections import Counter
from serann.engine.hip_engine import HipPopulationEngine
from serann.genome.interpreter import try_interpret
from serann.ops import hip_ops as H
irs=[try_interpret(s).ir for s in json.load(open('populations/bench_gen3_pop125.json'))][:125]
eng=HipPopulationEngine(irs, list(range(len(irs))), device="cpu")
mem=eng._alloc_buffers(750, with_grads=True)
pl=eng._build_plan("train",750,mem,[{"X":0,"g":0} for _ in irs],0,[0]*len(irs),None,adam_ctx=1)
L=[la for la in pl.launches if la.kind!="fn"]
fwd=pl.fwd_count
order=[None]*3+L[:fwd]+[None]+L[fwd:]
for i in map(int, sys.argv[1:]):
    la=order[i]
    d=np.frombuffer(la.descs.numpy().tobytes(), dtype=H.GEMM_DTYPE)
    c=Counter((int(r['M']),int(r['N']),int(r['K']),int(r['KH']),int(r['KW']),int(r['C']),int(r['flags'])) for r in d)
    print(i, la.arg, la.n, 'blocks', len(d), 'problems')
    for k,v in c.most_common(12): print('   M,N,K,KH,KW,C,flags', k, 'x', v)
