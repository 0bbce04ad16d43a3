"""Diagnostic (round 4, the r3 SIGSEGV): does torch keep using a HIP stream it did not create --
wrapped in torch.cuda.ExternalStream, as the dropped "partial" mode wrapped the engine's stream --
after the stream's owner destroyed it?  One mode per process:

  python3 tools/extstream_teardown.py owner_last    # tensors freed, group destroyed, then the stream
  python3 tools/extstream_teardown.py owner_first   # the stream destroyed while torch still holds
                                                    # the all-gather's tensors/work on it (what the
                                                    # test loop did when it rebound the Forest)
  python3 tools/extstream_teardown.py owner_sync    # owner_first after torch.cuda.synchronize() and
                                                    # freeing the tensors, group still alive
Prints "ok MODE" when the process reaches its end; a crash shows as the exit status.
"""
import ctypes
import os
import sys

import torch
import torch.distributed as dist

mode = sys.argv[1]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
# the HIP runtime torch loaded (one per process: the engine reuses it by SONAME)
path = [ln.split()[-1] for ln in open(f"/proc/{os.getpid()}/maps") if "libamdhip64" in ln][0]
hip = ctypes.CDLL(path)
s = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(s)) == 0
ext = torch.cuda.ExternalStream(s.value)
x = torch.ones(2, dtype=torch.float64, device="cuda")
with torch.cuda.stream(ext):
    out = torch.empty(2, dtype=torch.float64, device="cuda")   # a block of the caching allocator on ext
    for _ in range(50):
        dist.all_gather_into_tensor(out, x)
    y = out * 2
torch.cuda.synchronize()
print("gathered", float(y.sum()), flush=True)
if mode == "owner_last":
    del out, y
    torch.cuda.synchronize()
    dist.destroy_process_group()
    torch.cuda.empty_cache()
    assert hip.hipStreamDestroy(s) == 0
elif mode == "owner_first":
    assert hip.hipStreamDestroy(s) == 0
    del out, y
    dist.destroy_process_group()
    torch.cuda.empty_cache()
elif mode == "owner_sync":
    del out, y
    torch.cuda.synchronize()
    assert hip.hipStreamDestroy(s) == 0
    z = torch.ones(4, device="cuda") * 3        # the allocator reuses blocks after the stream is gone
    torch.cuda.synchronize()
    dist.destroy_process_group()
    torch.cuda.empty_cache()
print("ok", mode, flush=True)
