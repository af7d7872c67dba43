"""``ray_amd.util.pdb`` = the remote debugger (reference exposes ``ray.util.pdb``)."""

from ray_amd.util.rpdb import (RemotePdb, connect_pdb_client, list_breakpoints,  # noqa: F401
                               post_mortem, set_trace)
