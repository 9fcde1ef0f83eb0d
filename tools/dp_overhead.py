"""Config 4 overhead on one GPU (bs = 256 pairs, fp32, full fine-tune): ms/step of
  graph  — the captured step replayed (the N = 1 bench path),
  eager  — eager steps, two encoder streams, no DP,
  dp     — eager steps with the overlapped gradient all-reduce active on RCCL (ProcessGroupNCCL with
           one rank, mmfd.dp.GradAllReduce(force=True), default 32 MB per-stream buckets: packing,
           all_reduce calls, finish() wait + unpack — everything a rank does except the xGMI transfer),
  dp_graph — the same DP step captured as one HIP graph (the N > 1 bench path since round 4).
  python tools/dp_overhead.py [steps]"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd.dataset import synthetic_batch  # noqa: E402
from mmfd.dp import GradAllReduce  # noqa: E402
from mmfd.train import build_flagship  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
batch = synthetic_batch(256, seed=1000, device=dev)


def timed(fn, n):
    fn()
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / n


res = {}
tr = build_flagship(dev, "fp32", seed=42)
res["eager"] = timed(lambda: tr.step(batch), steps)
tr.capture(batch, warmup=1)
res["graph"] = timed(tr.replay, steps)
tr.release_graph()
del tr
torch.cuda.empty_cache()
dp = GradAllReduce(force=True)
tr = build_flagship(dev, "fp32", seed=42, dp=dp)
res["dp"] = timed(lambda: tr.step(batch), steps)
nb = dict(dp.last_buckets)
tr.capture(batch, warmup=1)
res["dp_graph"] = timed(tr.replay, steps)
tr.release_graph()
print({k: round(v, 1) for k, v in res.items()}, "buckets per stream:", nb, flush=True)
print(f"DP bookkeeping + RCCL calls: {res['dp'] - res['eager']:+.1f} ms/step over eager; eager over graph: "
      f"{res['eager'] - res['graph']:+.1f} ms/step; captured DP step over graph: "
      f"{res['dp_graph'] - res['graph']:+.1f} ms/step ({100 * (res['dp_graph'] / res['graph'] - 1):+.2f} %)", flush=True)
dist.destroy_process_group()
