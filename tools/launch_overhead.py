"""Per-kernel overhead of back-to-back launches inside a captured HIP graph.

Captures K tiny kernels (in-place add on a 256-float tensor) and times replays.
"""
import torch


def main():
    x = torch.zeros(256, device="cuda")
    big = torch.zeros(32768 * 64, device="cuda")
    for name, t in (("tiny", x), ("8MB", big)):
        for K in (1, 10, 40):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    t.add_(1.0)
                with torch.cuda.graph(g, stream=s):
                    for _ in range(K):
                        t.add_(1.0)
            torch.cuda.current_stream().wait_stream(s)
            for _ in range(10):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            reps = 200
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            print(f"{name:5s} K={K:3d}: {us:8.2f} us per replay, {us / K:6.2f} us per kernel")


if __name__ == "__main__":
    main()
