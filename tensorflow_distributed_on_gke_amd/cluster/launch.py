"""Per-node process launcher: one training process per GPU.

Spawns `nproc` children (subprocesses, never exec) with the env:// variables
for this node, forwards their output, and implements failure detection: if
any child exits non-zero, the others are terminated and the launcher exits
with that child's code (so a Kubernetes pod restarts as a unit; the reference
relied on the StatefulSet restarting a dead pod, cluster.py / running.md).
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from typing import List, Optional

from tensorflow_distributed_on_gke_amd.cluster.rendezvous import ClusterSpec, export_env


def launch(argv: List[str], nproc: int, spec: ClusterSpec, poll_s: float = 0.5,
           env_extra: Optional[dict] = None) -> int:
    procs = []
    for lr in range(nproc):
        env = dict(os.environ)
        saved = dict(os.environ)
        export_env(spec, nproc, lr)
        env.update({k: os.environ[k] for k in ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "RANK",
                                               "LOCAL_RANK", "LOCAL_WORLD_SIZE", "NODE_RANK")})
        os.environ.clear()
        os.environ.update(saved)
        env.pop("THIS_POD_NAME", None)  # children must not re-run discovery
        if "OMP_NUM_THREADS" not in os.environ:
            # CPU (gloo) runs: split the host's cores between the ranks
            env["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // nproc))
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable] + argv, env=env, start_new_session=True))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0:
                    rc = r
                    for q in procs:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
                    deadline = time.time() + 30
                    for q in procs:
                        try:
                            q.wait(timeout=max(0.1, deadline - time.time()))
                        except subprocess.TimeoutExpired:
                            os.killpg(q.pid, signal.SIGKILL)
                    procs = []
                    break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for q in procs:
            os.killpg(q.pid, signal.SIGTERM)
        rc = 130
    return rc
