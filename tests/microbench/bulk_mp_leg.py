"""Test infrastructure: bench.py's bulk_multipage writer leg alone (C2 Rec8, 1 MiB pages, 128 MiB
row groups), for kernel traces:
  rocprofv3 --kernel-trace --stats -d gpurun_out/bmp -- python3 tests/microbench/bulk_mp_leg.py [records] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kafka-parquet-writer_amd"), os.path.join(ROOT, "synth")]
import bench  # noqa: E402
import kpw  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
kind, _, seed, _ = bench.WORKLOADS["c2"][:4]
print(bench.writer_leg(kpw, kind, seed, n, 0, steps, 1, page_size=bench.MiB), flush=True)
