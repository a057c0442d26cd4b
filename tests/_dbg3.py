import sys, numpy as np
sys.path.insert(0,'.')
import pacmann_amd as pm
from oracle import oracle as O
N,E,B,n,dup = int(sys.argv[1]),int(sys.argv[2]),int(sys.argv[3]),int(sys.argv[4]),int(sys.argv[5])
db=np.random.default_rng(N+E).integers(0,2**64,size=N*E,dtype=np.uint64)
g=pm.SimpleBatchPianoPIR(N,E*8,B,db,8,seed=20240501)
o=O.SimpleBatchPianoPIR(N,E*8,B,db,8,seed=20240501)
g.Preprocessing(); o.Preprocessing()
rng=np.random.default_rng(N)
for b in range(5):
    q=rng.choice(N,size=n,replace=False).astype(np.uint64)
    if dup: q[7::11]=q[1]
    got,_=g.Query(q); want,_=o.Query(q)
    assert np.array_equal(got,want), b
print('ok',sys.argv[1:],flush=True)
