"""Do two HIP streams run kernels concurrently on this box?  (run on the GPU box)

Stream A: a ~200 us compute kernel (fp32 matmul); stream B: torch.cuda._sleep
(one spinning wave).  Prints each alone and both together: together ~= max
means concurrent, ~= sum means serialised.  Variants: B at high priority,
B created before / after A, the legacy null stream as A.
"""
import time

import torch


def timed(fn, reps=20):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record(torch.cuda.default_stream())
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    out = torch.empty(4096, 4096, device=dev)
    # cycles for ~100 us of sleep at ~100 MHz s_memrealtime? calibrate
    sA_opts = {"side": torch.cuda.Stream(device=dev), "null": torch.cuda.default_stream(dev)}
    for prio in (0, -1):
        sB = torch.cuda.Stream(device=dev, priority=prio)
        for name, sA in sA_opts.items():
            def comp():
                with torch.cuda.stream(sA):
                    for _ in range(4):
                        torch.mm(a, b, out=out)

            def slp():
                with torch.cuda.stream(sB):
                    torch.cuda._sleep(2_000_000)

            def both():
                comp()
                slp()

            def join():
                torch.cuda.current_stream().wait_stream(sA)
                torch.cuda.current_stream().wait_stream(sB)

            tc = timed(lambda: (comp(), join()))
            ts = timed(lambda: (slp(), join()))
            tb = timed(lambda: (both(), join()))
            print(f"A={name:4s} B priority {prio:2d}: compute {tc:.3f} ms, sleep {ts:.3f} ms, both {tb:.3f} ms "
                  f"-> {'concurrent' if tb < 0.8 * (tc + ts) else 'SERIAL'}", flush=True)


if __name__ == "__main__":
    main()
