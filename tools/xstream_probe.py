"""Cost of a cross-stream dependency on this ROCm stack: per iteration a tiny
kernel on the main stream, an event, the side stream waiting on it and running a tiny kernel,
an event back, the main stream waiting -- against the same kernels on one stream.  1,000
iterations queued without host synchronisation; wall time per iteration."""
import sys
import time

import torch


def run(mode, n=1000, prio=0):
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream(priority=prio)
    x = torch.zeros(1, device="cuda")
    y = torch.zeros(1, device="cuda")
    e1 = torch.cuda.Event()
    e2 = torch.cuda.Event()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        x.add_(1)
        if mode == "one":
            y.add_(1)
            x.add_(1)
        else:
            e1.record(s1)
            s2.wait_event(e1)
            with torch.cuda.stream(s2):
                y.add_(1)
            e2.record(s2)
            if mode == "two":
                x.add_(1)
            s1.wait_event(e2)
            if mode == "two_after":
                x.add_(1)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    for rep in range(2):
        for mode in ("one", "two", "two_after"):
            for prio in (0, -1):
                print("rep {} {:10s} prio {:2d}: {:.1f} us/iter".format(rep, mode, prio, run(mode, prio=prio)),
                      flush=True)


if __name__ == "__main__":
    sys.exit(main())
