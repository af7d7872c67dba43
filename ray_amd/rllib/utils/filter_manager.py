"""``FilterManager`` (reference: python/ray/rllib/utils/filter_manager.py): merge the
buffered statistics of remote copies of observation filters into the local ones and push
the result back."""

from __future__ import annotations


class FilterManager:
    @staticmethod
    def synchronize(local_filters: dict, worker_set_or_filters, update_remote: bool = True,
                    timeout_seconds=None, use_remote_data_for_update: bool = True):
        """``worker_set_or_filters``: a list of {name: Filter} dicts (the remote copies'
        buffers), or an object with ``foreach_env_runner(fn)`` returning them."""
        remotes = worker_set_or_filters
        if hasattr(remotes, "foreach_env_runner"):
            remotes = remotes.foreach_env_runner(lambda w: getattr(w, "filters", {}))
        for rf in remotes or []:
            if use_remote_data_for_update:
                for k, f in rf.items():
                    if k in local_filters:
                        local_filters[k].apply_changes(f, with_buffer=False)
        if update_remote:
            for rf in remotes or []:
                for k in rf:
                    if k in local_filters:
                        rf[k].sync(local_filters[k])
                        rf[k].reset_buffer()
        return local_filters
