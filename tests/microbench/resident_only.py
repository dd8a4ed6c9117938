"""Test infrastructure: the bench's resident leg alone (kpw_encoder_encode on a C2 batch already
in HBM, one encoder, 3 timed encodes), for kernel traces without the writer's concurrency:
  rocprofv3 --kernel-trace --stats -d gpurun_out/res -- python3 tests/microbench/resident_only.py [workload]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kafka-parquet-writer_amd"), os.path.join(ROOT, "synth")]
import bench  # noqa: E402
import kpw  # noqa: E402
import synth  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
kind, n, seed, _ = bench.WORKLOADS[wl][:4]
schema_s = synth.SCHEMAS[kind]
schema = kpw.Schema(schema_s.message_name, schema_s.columns, schema_s.proto_class)
batches = [synth.generate(kind, seed + 0x1000 * k, n) for k in range(2)]
r = bench.resident_encode(kpw, schema, batches, 0)
print(r)
