import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_ccrdt_amd.engine import DeviceTrmvBatch, TopkRmvEngine, gen_trmv
nk, n_ops = 1 << 20, 100_000_000
eng = TopkRmvEngine(nk, 100, 8)  # (CCRDT_LIB selects the build)
for i in range(4):
    b = gen_trmv(n_ops, nk, 8, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64, seed=0xCC0DE + 2 + 7919 * i, clock0=i * n_ops)
    db = DeviceTrmvBatch(b); del b
    eng.apply_device(db); eng.sync(); db.close()
    print(os.environ.get("CCRDT_LIB", "default"), "batch", i + 1, "chain ms", round(eng.last_kernel_ms(), 2), flush=True)
