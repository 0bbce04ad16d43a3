"""A/B of armed objective calls (ggp_arm) on the C2 forest (1000 trees x 200 rows: 2000 paths): blocks of
chained calls on one handle, armed and plain in turn, each block after settling calls; per-call
wall time (mean and median) and the handle's armed-call count"""
import statistics
import sys
import time

sys.path.insert(0, ".")
import gfp_gaussian_process_amd as g  # noqa: E402
from bench import P_EXAMPLE  # noqa: E402


def block(f, n):
    t = [0.0] * (n + 1)
    t[0] = time.perf_counter()
    for k in range(n):
        f.total_likelihood(P_EXAMPLE)
        t[k + 1] = time.perf_counter()
    return [1e6 * (b - a) for a, b in zip(t, t[1:])]


def main():
    f = g.Forest(g.HostForest.synthetic(int(sys.argv[1]) if len(sys.argv) > 1 else 1000, 200))
    for _ in range(500):
        f.total_likelihood(P_EXAMPLE)
    res = {0: [], 1: []}
    for rep in range(3):
        for on in (0, 1):
            f.arm(bool(on))
            for _ in range(300):
                f.total_likelihood(P_EXAMPLE)
            a0 = f.arm(None)
            us = block(f, 2000)
            a1 = f.arm(None)
            res[on].append((statistics.mean(us), statistics.median(us), a1 - a0))
            tr = f.call_trace(512)   # (enqueue_us, wait_us, result_us, kernel_us, shader_mhz, call)
            med = [statistics.median(tr[:, j]) for j in range(5)]
            print(f"rep {rep} arm {on}: mean {statistics.mean(us):.2f} us median {statistics.median(us):.2f} us "
                  f"armed {a1 - a0}; trace medians enq {med[0]:.2f} wait {med[1]:.2f} res {med[2]:.2f} "
                  f"kern {med[3]:.2f} mhz {med[4]:.0f}", flush=True)
    f.arm(False)
    for on in (0, 1):
        m = [x[0] for x in res[on]]
        md = [x[1] for x in res[on]]
        print(f"arm {on}: mean of means {statistics.mean(m):.2f} us, median of medians {statistics.median(md):.2f} us")
    print("total", f.total_likelihood(P_EXAMPLE))


if __name__ == "__main__":
    main()
