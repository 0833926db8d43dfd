"""Kubernetes StatefulSet discovery -> torch.distributed rendezvous.

Reference: distributed_training_transformer/cluster/cluster.py:12-109
(TensorflowKubernetesCluster): the pod ordinal comes from THIS_POD_NAME
("<statefulset>-<ordinal>"), peers are found by polling the K8s API every 2 s
until `worker_count` pods of the set have IPs, a heartbeat barrier follows,
then TF_CONFIG + MultiWorkerMirroredStrategy. Here the result is an env://
rendezvous for torch.distributed (MASTER_ADDR = pod 0's IP) and one process per
GPU inside each pod.

Fixes two reference bugs: pods are matched on the full
StatefulSet name (`rsplit('-', 1)`, not the first dash token) and ordered by
numeric ordinal (the reference sorted names lexicographically, so with >= 10
pods "x-10" < "x-2" disagreed with the task index).

The API client is a minimal in-cluster REST client (service-account token +
CA bundle); tests inject a fake `list_pods` callable.
"""
from __future__ import annotations

import json
import os
import ssl
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple
from urllib.request import Request, urlopen

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


@dataclass
class PodInfo:
    name: str
    ip: Optional[str]


def parse_pod_name(pod_name: str) -> Tuple[str, int]:
    base, _, ordinal = pod_name.rpartition("-")
    if not base or not ordinal.isdigit():
        raise ValueError(f"pod name {pod_name!r} is not <statefulset>-<ordinal>")
    return base, int(ordinal)


def incluster_list_pods(namespace: str = "default") -> List[PodInfo]:  # pragma: no cover - needs a cluster
    host = os.environ["KUBERNETES_SERVICE_HOST"]
    port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
    token = open(os.path.join(SA_DIR, "token")).read().strip()
    ctx = ssl.create_default_context(cafile=os.path.join(SA_DIR, "ca.crt"))
    req = Request(f"https://{host}:{port}/api/v1/namespaces/{namespace}/pods",
                  headers={"Authorization": f"Bearer {token}"})
    with urlopen(req, context=ctx, timeout=10) as r:
        items = json.loads(r.read().decode())["items"]
    return [PodInfo(i["metadata"]["name"], i.get("status", {}).get("podIP")) for i in items]


def discover_peers(pod_name: str, worker_count: int,
                   list_pods: Callable[[], Sequence[PodInfo]],
                   poll_s: float = 2.0, timeout_s: Optional[float] = None,
                   verbose: bool = False) -> List[str]:
    """IPs of the StatefulSet's pods, ordered by ordinal, once all
    `worker_count` of them are scheduled with an IP."""
    base, _ = parse_pod_name(pod_name)
    if verbose:
        print(f"Waiting until {worker_count - 1} peers become available.")
    deadline = None if timeout_s is None else time.time() + timeout_s
    while True:
        workers = []
        for pod in list_pods():
            try:
                b, ordinal = parse_pod_name(pod.name)
            except ValueError:
                continue
            if b == base and pod.ip:
                workers.append((ordinal, pod))
        if len(workers) == worker_count:
            break
        if deadline is not None and time.time() > deadline:
            raise TimeoutError(f"found {len(workers)}/{worker_count} pods of {base}")
        time.sleep(poll_s)
    workers.sort(key=lambda t: t[0])
    ordinals = [o for o, _ in workers]
    if ordinals != list(range(worker_count)):
        raise RuntimeError(f"unexpected StatefulSet ordinals {ordinals}")
    if verbose:
        print("Found pods in stateful set:")
        for _, pod in workers:
            print(pod.name + " " + pod.ip)
    return [pod.ip for _, pod in workers]
