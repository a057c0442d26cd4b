# Diagnostic: per-phase s_memtime stamps of k_resolve.  Build the PM_STAMPS
# variant (pacmann_amd/libpacmann_stamps.so) and run with
# PM_LIB=pacmann_amd/libpacmann_stamps.so python tools/probe_resolve_stamps.py
import sys, time, numpy as np
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__file__), '..'))
import pacmann_amd as pm
N,E,B=1_000_000,80,32
db=np.random.default_rng(0).integers(0,2**64,size=N*E,dtype=np.uint64)
g=pm.SimpleBatchPianoPIR(N,E*8,B,db,8,seed=1)
g.Preprocessing()
rng=np.random.default_rng(1)
qs=rng.integers(0,N,size=(400,96)).astype(np.uint64)
t=time.time()
for q in qs: g.Query(q)
print('per step us', (time.time()-t)/len(qs)*1e6, flush=True)
del g
