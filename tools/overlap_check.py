"""bench.py's pipelined N > 1 step checked on one GPU: the same stream pattern (two extractors'
output buffers alternating, the all-gather of step i on a second stream beside step i + 1's
extraction, the extraction waiting on the device for the gather that last read its buffer) with an
RCCL group of one rank, every step gathered into its own output and compared bitwise with the
rows an eager launch gives for that step's batch.  Three distinct batches rotate, so a gather that
read a buffer already overwritten by a later step shows up as a mismatch.
  python tools/overlap_check.py [clips] [K]"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dsp-audioreclabs_amd"))
import torch
import torch.distributed as dist
from src.pipeline import FeatureExtractor
from src.synth import make_batch_device

C = int(sys.argv[1]) if len(sys.argv) > 1 else 12500
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29534")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
P = 3
pool = [make_batch_device(C, dev, base_seed=p) for p in range(P)]
ref = FeatureExtractor(1102, 441, "hamming", True, device=dev)
want = [ref(b)["rows"].clone() for b in pool]
fxs = (FeatureExtractor(1102, 441, "hamming", True, device=dev), FeatureExtractor(1102, 441, "hamming", True, device=dev))
outs = [torch.empty((C, 19), dtype=torch.int32, device=dev) for _ in range(K)]
stream = torch.cuda.current_stream(dev)
comm = torch.cuda.Stream(dev)
works = [None, None]
torch.cuda.synchronize()
for i in range(K):
    j = i & 1
    if works[j] is not None:
        works[j].wait()
    rows = fxs[j](pool[i % P])["rows"]
    comm.wait_stream(stream)
    with torch.cuda.stream(comm):
        works[j] = dist.all_gather_into_tensor(outs[i], rows, async_op=True)
torch.cuda.synchronize()
bad = [i for i in range(K) if not torch.equal(outs[i], want[i % P])]
print(json.dumps({"clips": C, "steps": K, "batches": P, "steps_equal": K - len(bad), "bad_steps": bad}))
dist.destroy_process_group()
sys.exit(1 if bad else 0)
