"""Per-call cost of the sharded objective's collective (1-rank nccl group, one GPU): the
direct objective, the shipped ShardedObjective path (pinned staging) and the earlier form
(two element fills on the device tensor, blocking .cpu()), alternating blocks."""
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd.distributed import ShardedObjective, combine_partials  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
hf = g.HostForest.synthetic(1000, 200)
fd, fn, fo = g.Forest(hf), g.Forest(hf), g.Forest(hf)
new = ShardedObjective(fn, always_gather=True)
send = torch.zeros(2, dtype=torch.float64, device="cuda")
recv = torch.zeros(2, dtype=torch.float64, device="cuda")


def old(p):
    v = fo.total_likelihood(p)
    send[0] = v
    send[1] = 0.0
    dist.all_gather_into_tensor(recv, send)
    got = recv.cpu().numpy().reshape(1, 2)
    return combine_partials(got[:, 0], got[:, 1] != 0)[0]


res = {"direct": [], "pinned": [], "old": []}
for rep in range(5):
    for name, fnc in (("direct", fd.total_likelihood), ("pinned", new.total_likelihood), ("old", old)):
        for _ in range(10):
            fnc(P)
        t0 = time.perf_counter()
        for _ in range(100):
            fnc(P)
        res[name].append(1e3 * (time.perf_counter() - t0) / 100)
dist.destroy_process_group()
print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in res.items()}), json.dumps(res))
