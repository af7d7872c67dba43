"""One process-wide lock around HIP-graph capture. A capture in ``global`` mode makes any
other thread's synchronizing call in the same process fail, so the threads that share a
GPU context — the learner capturing its update graph and an in-process policy server
replaying its inference graph (rllib/env/policy_server.py) — take turns through it."""

import threading

CAPTURE_LOCK = threading.RLock()
