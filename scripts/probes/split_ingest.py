"""Where does the streaming_split -> GPU consumer path (the TorchTrainer data bench) spend
time? A 0.5-GPU consumer actor iterates its shard under cProfile."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import ray_amd as ray  # noqa: E402
import ray_amd.data as rd  # noqa: E402
from ray_amd.data import bench as db  # noqa: E402
from ray_amd.data.preprocessors import GPUImageNormalize  # noqa: E402


@ray.remote(num_gpus=0.5)
class Consumer:
    def run(self, it, warm, n):
        import torch

        dev = torch.device("cuda", 0)
        b = iter(it.iter_torch_batches(batch_size=256, device=dev, drop_last=True))
        for _ in range(warm):
            next(b)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        t0 = time.perf_counter()
        for _ in range(n):
            next(b)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(35)
        return n * 256 / dt, s.getvalue()


ray.init(num_cpus=16, num_gpus=1)
N = 70 * 256
for gpu in (False, True):
    ds = rd.range(N, override_num_blocks=70).map_batches(db._make_images, batch_size=256)
    if gpu:
        ds = GPUImageNormalize(out_dtype="bf16", batch_size=256, num_gpus=0.5,
                               keep_on_device=True).transform(ds)
    (it,) = ds.streaming_split(1)
    c = Consumer.remote()
    rate, prof = ray.get(c.run.remote(it, 5, 60))
    print("gpu stage" if gpu else "host blocks", "img/s", round(rate, 1), flush=True)
    print(prof, flush=True)
    ray.kill(c)
ray.shutdown()
