"""The bench's training step run eagerly with the two encoders (and the head's halves) on ONE stream,
for a kernel trace whose per-kernel durations are not stretched by a concurrent stream:
  rocprofv3 --kernel-trace --stats -d gpurun_out/serial -o run --output-format csv -- \\
      python3 tools/serial_step.py [fp32|bf16] [steps]
then python3 tools/step_breakdown.py gpurun_out/serial/run_kernel_stats.csv (steps = AdamW launches)."""
import os
import sys

os.environ["MMFD_SERIAL_HEAD"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mmfd.dataset import synthetic_batch  # noqa: E402
from mmfd.train import build_flagship  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    tr = build_flagship(dev, prec, dropout=0.1, seed=42, rank=0)
    tr.concurrent = False
    batch = synthetic_batch(256, seed=1000, device=dev)
    tr.step(batch)  # warm-up (allocator, kernel attributes)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        tr.step(batch)
    e1.record()
    torch.cuda.synchronize()
    print(f"{prec}: serialized eager step {e0.elapsed_time(e1) / steps:.1f} ms ({steps} steps after 1 warm-up)")


if __name__ == "__main__":
    main()
