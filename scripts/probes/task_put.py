import sys, time
sys.path.insert(0, ".")
import numpy as np
from ray_amd.data import bench as db
import ray_amd as ray
from ray_amd._private import serialization as ser
ray.init(num_cpus=16)
@ray.remote
def mk(i):
    t0=time.perf_counter()
    b = db._make_images({"id": np.arange(256)+i})
    t1=time.perf_counter()
    s = ser.serialize(b, None)
    t2=time.perf_counter()
    r = ray.put(b)
    t3=time.perf_counter()
    return (t1-t0, t2-t1, t3-t2), r
for n in (1, 16, 16, 64):
    t0=time.perf_counter(); r=ray.get([mk.remote(i) for i in range(n)]); dt=time.perf_counter()-t0
    print(n, "tasks: ms/task", round(dt/n*1e3,2), "make/ser/put ms", np.round(np.mean([x[0] for x in r],0)*1e3,2), flush=True)
    del r
ray.shutdown()
