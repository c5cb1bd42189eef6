import numpy as np, torch, sys
sys.path.insert(0, '.')
from tests.conftest import CONFIGS
from tests.test_gpu_parity import VK, _engine, _oracle
cfg = CONFIGS["hist_256_c16"]
o = _oracle(cfg)
for fuse, fuse_seg in ((1, 1), (1, 0), (0, 1)):
  for n in (1024,):
    eng = _engine(cfg); eng.set_option("fuse_acc", fuse)
    d = o.gen_reports(VK, n, seed=1, n_threads=8)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    msgs = torch.zeros((n, 16), dtype=torch.uint8, device=dev); status = torch.zeros(n, dtype=torch.uint8, device=dev)
    agg = torch.zeros((1, 4096), dtype=torch.uint8, device=dev); cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    seg = t(np.zeros(n, np.uint32)) if fuse_seg else None
    eng.prepare_aggregate_device(t(d["nonces"]), t(d["public_shares"]), t(d["helper_shares"]), t(d["leader_prep_shares"]), seg, 1, msgs, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    bad = np.nonzero(st)[0]
    print("fuse", fuse, "seg", fuse_seg, "n", n, "bad count", len(bad), "bad waves", sorted(set((bad // 64).tolist()))[:20], "lanes", sorted(set((bad % 64).tolist()))[:8])
