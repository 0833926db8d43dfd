"""Cluster bootstrap: decide this process's (node, rank, world) and the
rendezvous address, in local or Kubernetes mode.

Local mode (THIS_POD_NAME unset; reference cluster.py:35-40): a single node;
WORLD_SIZE/RANK come from the launcher (torch.distributed.run or our
`launch`), default 1 process.

Kubernetes mode (THIS_POD_NAME set; reference cluster.py:41-66): node rank =
pod ordinal, peers from the API (k8s.discover_peers), heartbeat barrier
(heartbeat.wait_for_cluster), MASTER_ADDR = pod 0's IP. The reference's fixed
10 s sleep for non-chief pods is replaced by the TCPStore rendezvous, which
blocks until the chief's store is up.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

from tensorflow_distributed_on_gke_amd.cluster import heartbeat, k8s


@dataclass
class ClusterSpec:
    node_rank: int
    num_nodes: int
    node_ips: List[str]
    master_addr: str
    master_port: int
    heartbeat: Optional[heartbeat.HeartbeatServer] = None

    @property
    def chief(self) -> bool:
        return self.node_rank == 0


def bootstrap(worker_count: int, namespace: str = "default", heartbeat_port: int = 3479,
              master_port: int = 3480, verbose: bool = False,
              list_pods: Optional[Callable[[], Sequence[k8s.PodInfo]]] = None,
              heartbeat_timeout_s: Optional[float] = 600.0) -> ClusterSpec:
    pod = os.environ.get("THIS_POD_NAME")
    if not pod:
        if verbose:
            print("Environment variable THIS_POD_NAME not set, running in local mode.", flush=True)
        return ClusterSpec(0, 1, ["127.0.0.1"], os.environ.get("MASTER_ADDR", "127.0.0.1"),
                           int(os.environ.get("MASTER_PORT", master_port)))
    _, ordinal = k8s.parse_pod_name(pod)
    if verbose:
        print("Pod name from environment variable: " + pod)
    ips = k8s.discover_peers(pod, worker_count, list_pods or (lambda: k8s.incluster_list_pods(namespace)),
                             verbose=verbose)
    hb = heartbeat.wait_for_cluster(ips, heartbeat_port, verbose=verbose, timeout_s=heartbeat_timeout_s)
    return ClusterSpec(ordinal, worker_count, ips, ips[0], master_port, hb)


def export_env(spec: ClusterSpec, nproc_per_node: int, local_rank: int) -> None:
    """torch.distributed env:// variables for one process of this node."""
    os.environ["MASTER_ADDR"] = spec.master_addr
    os.environ["MASTER_PORT"] = str(spec.master_port)
    os.environ["WORLD_SIZE"] = str(spec.num_nodes * nproc_per_node)
    os.environ["RANK"] = str(spec.node_rank * nproc_per_node + local_rank)
    os.environ["LOCAL_RANK"] = str(local_rank)
    os.environ["LOCAL_WORLD_SIZE"] = str(nproc_per_node)
    os.environ["NODE_RANK"] = str(spec.node_rank)
