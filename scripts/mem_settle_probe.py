"""Free-HBM timeline right after another process exits: prints torch.cuda.mem_get_info()
every 0.5 s (checks whether the previous process's memory returns to the pool gradually,
which would explain a slow window after big processes exit)."""

import json
import sys
import time

import torch


def main(duration=40.0):
    t0 = time.time()
    torch.cuda.init()
    while time.time() - t0 < duration:
        free, total = torch.cuda.mem_get_info()
        print(json.dumps({"t": round(time.time() - t0, 1), "free_gb": round(free / 2**30, 1),
                          "total_gb": round(total / 2**30, 1)}), flush=True)
        time.sleep(0.5)


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 40.0)
