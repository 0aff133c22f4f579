"""Per-kernel floor on this box: N tiny dependent kernels, eager vs HIP graph."""
import time

import torch


def run(fn, n_iter=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n_iter):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n_iter


def main():
    x = torch.zeros(1024, device="cuda")
    big = torch.zeros(64 << 20, device="cuda")
    K = 200

    def chain():
        for _ in range(K):
            x.add_(1.0)

    def chain_big():
        for _ in range(K // 10):
            big.add_(1.0)
            for _ in range(9):
                x.add_(1.0)

    for name, f in (("tiny", chain), ("mixed", chain_big)):
        f()
        e = run(f)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            f()
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                f()
        torch.cuda.current_stream().wait_stream(s)
        gr = run(g.replay)
        print(f"{name}: eager {e / K * 1e6:.2f} us/kernel, graph {gr / K * 1e6:.2f} us/kernel", flush=True)


if __name__ == "__main__":
    main()
