"""Ray Client: drive a cluster from another process / host over TCP
(reference: python/ray/util/client/{__init__,worker,server/server}.py).

``ray_amd.init("ray://host:port")`` installs a ``ClientCoreWorker`` as the process'
core worker, so the whole public API (tasks, actors, put/get/wait, named actors,
kill/cancel, cluster info) works unchanged; every call is forwarded to a client
server (``python -m ray_amd.util.client.server``), which is a real driver of the
cluster and holds the server-side ObjectRefs / ActorHandles on the client's behalf.
Object references cross the wire by id (pickle persistent ids), so refs nested in
task arguments or in returned values stay refs; the client's reference counts
release the server-side refs when they drop to zero."""

from ray_amd.util.client.worker import ClientCoreWorker  # noqa: F401

DEFAULT_PORT = 10001
