"""Two-stream concurrency probe: each second, time (a) two GEMMs + an elementwise chain on
ONE stream, (b) the same split over two streams with cross-stream event waits (the shape
of the GPT-2 step's side-stream weight gradients). Prints one JSON line per sample."""

import json
import time

import torch


def main(duration=45.0):
    dev = torch.device("cuda")
    a = torch.randn(8192, 768, device=dev).bfloat16()
    w = torch.randn(3072, 768, device=dev).bfloat16()
    g = torch.randn(8192, 3072, device=dev).bfloat16()
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def serial():
        for _ in range(20):
            y = a @ w.t()
            y.mul_(1.0001)
            z = g.t() @ a
            z.add_(1.0)

    def split():
        for _ in range(20):
            y = a @ w.t()
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                z = g.t() @ a
                z.add_(1.0)
            y.mul_(1.0001)
            main_s.wait_stream(side)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    timed(serial)
    timed(split)
    t0 = time.time()
    while time.time() - t0 < duration:
        s = timed(serial)
        p = timed(split)
        print(json.dumps({"t": round(time.time() - t0, 1), "serial_ms": round(s, 2),
                          "two_stream_ms": round(p, 2)}), flush=True)
        time.sleep(1.0)


if __name__ == "__main__":
    main()
