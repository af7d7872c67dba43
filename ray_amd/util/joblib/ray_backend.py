"""joblib ParallelBackend that runs each batch of calls as a ray_amd task."""

from __future__ import annotations

from joblib._parallel_backends import AutoBatchingMixin, ParallelBackendBase

import ray_amd as ray


def _run_batch(batch):
    return batch()


class RayBackend(AutoBatchingMixin, ParallelBackendBase):
    """Batches are ``@ray.remote`` tasks; results come back through ObjectRef futures.

    ``ray_remote_args`` (backend kwarg) are the task options, e.g.
    ``parallel_backend("ray", ray_remote_args={"num_cpus": 2})``. ``n_jobs=-1`` means the
    cluster's CPU count divided by the CPUs each task asks for."""

    supports_retrieve_callback = True
    supports_inner_max_num_threads = False
    default_n_jobs = -1

    def __init__(self, nesting_level=None, inner_max_num_threads=None, ray_remote_args=None,
                 **kwargs):
        super().__init__(nesting_level=nesting_level,
                         inner_max_num_threads=inner_max_num_threads, **kwargs)
        self._remote_args = dict(ray_remote_args or {})
        self._remote_args.setdefault("num_cpus", 1)
        self._task = None
        self._pending: dict = {}

    def effective_n_jobs(self, n_jobs):
        if n_jobs == 0:
            raise ValueError("n_jobs == 0 in Parallel has no meaning")
        if n_jobs is None or n_jobs < 0:
            if not ray.is_initialized():
                ray.init()
            cpus = float(ray.cluster_resources().get("CPU", 1))
            per = float(self._remote_args.get("num_cpus") or 1) or 1.0
            slots = max(1, int(cpus // per))
            return slots if n_jobs is None else max(1, slots + 1 + n_jobs)  # -1: all, -2: all but one
        return n_jobs

    def configure(self, n_jobs=1, parallel=None, **backend_args):
        if not ray.is_initialized():
            ray.init()
        self.parallel = parallel
        self._task = ray.remote(**self._remote_args)(_run_batch)
        return self.effective_n_jobs(n_jobs)

    def submit(self, func, callback=None):
        ref = self._task.remote(func)
        fut = ref.future()
        self._pending[id(fut)] = ref
        fut.add_done_callback(lambda f: self._pending.pop(id(f), None))
        if callback is not None:
            fut.add_done_callback(callback)
        return fut

    def retrieve_result_callback(self, future):
        return future.result()

    def abort_everything(self, ensure_ready=True):
        for ref in list(self._pending.values()):
            try:
                ray.cancel(ref, force=True)
            except Exception:
                pass
        self._pending.clear()
        if ensure_ready:
            self.configure(n_jobs=self.parallel.n_jobs if self.parallel else 1,
                           parallel=self.parallel)

    def terminate(self):
        self._pending.clear()

    def get_nested_backend(self):
        from joblib._parallel_backends import SequentialBackend

        return SequentialBackend(nesting_level=(self.nesting_level or 0) + 1), None
