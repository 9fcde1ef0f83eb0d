"""Repeat the world-1 RCCL graph-captured DP step test N times in one process (diagnosing an
intermittent ProcessGroupNCCL watchdog failure: hipErrorCapturedEvent).
    python tools/dp_graph_repeat.py N"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import test_dp_gpu as T  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ok = 0
    for i in range(n):
        t0 = time.time()
        try:
            T.test_dp_nccl_world1_graph_captured_step()
            ok += 1
            print(f"run {i}: ok ({time.time() - t0:.0f} s)", flush=True)
        except BaseException as e:  # noqa: BLE001
            print(f"run {i}: FAILED ({time.time() - t0:.0f} s): {str(e)[:300]}", flush=True)
    print(f"{ok}/{n} passed (TORCH_NCCL_CUDA_EVENT_CACHE={os.environ.get('TORCH_NCCL_CUDA_EVENT_CACHE')}, "
          f"MMFD_DP_QUIESCE={os.environ.get('MMFD_DP_QUIESCE')})", flush=True)


if __name__ == "__main__":
    main()
