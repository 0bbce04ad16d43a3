"""NodeExchange latency (diagnostic, CPU only): python tools/node_exchange_bench.py WORLD
WORLD processes on this host exchange 16 B each through host shared memory (distributed.NodeExchange),
then through gloo's all_gather_into_tensor; microseconds per call on every rank."""
import os, sys, time, socket
import numpy as np
import torch.multiprocessing as mp
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

def w(rank, world, port, q):
    import torch, torch.distributed as dist
    from gfp_gaussian_process_amd.distributed import NodeExchange
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    x = NodeExchange(dist, None, 2)
    for _ in range(200): x.exchange((1.0, 0.0))
    n = 5000
    t0 = time.perf_counter()
    for k in range(n): x.exchange((float(k), 0.0))
    t_x = (time.perf_counter() - t0) / n
    s = torch.zeros(2, dtype=torch.float64); r = torch.zeros(2 * world, dtype=torch.float64)
    for _ in range(50): dist.all_gather_into_tensor(r, s)
    t0 = time.perf_counter()
    for k in range(500): dist.all_gather_into_tensor(r, s)
    t_g = (time.perf_counter() - t0) / 500
    x.close()
    q.put((rank, t_x * 1e6, t_g * 1e6))
    dist.destroy_process_group()

if __name__ == "__main__":
    world = int(sys.argv[1])
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn"); q = ctx.Queue()
    ps = [ctx.Process(target=w, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=300) for _ in range(world))
    [p.join() for p in ps]
    print(world, "shm us/call", [round(a[1], 2) for a in res], "gloo us/call", [round(a[2], 1) for a in res])
