import numpy as np, time, scipy.linalg.lapack as L
from threadpoolctl import threadpool_limits
rng=np.random.default_rng(0)
H=np.triu(rng.standard_normal((128,128)),-1)
def best(f, n=15):
    b=1e9
    for _ in range(n):
        t=time.perf_counter(); f(); b=min(b,time.perf_counter()-t)
    return b*1e3
with threadpool_limits(1):
    print("scipy dgeev 4n", best(lambda: L.dgeev(H, compute_vl=0, lwork=512)))
    print("numpy eig", best(lambda: np.linalg.eig(H)))
    print("scipy dgeev novec", best(lambda: L.dgeev(H, compute_vl=0, compute_vr=0)))
    print("numpy eigvals", best(lambda: np.linalg.eigvals(H)))
