"""Cluster layer: heartbeat barrier, Kubernetes discovery (fake API), rendezvous
env, launcher failure detection. CPU only."""
import os
import sys
import time

import pytest

from tensorflow_distributed_on_gke_amd.cluster import heartbeat, k8s, launch, rendezvous


def test_heartbeat_barrier_and_probe():
    a = heartbeat.start_heartbeat_server(0)
    b = heartbeat.start_heartbeat_server(0)
    try:
        assert heartbeat.probe("127.0.0.1", a.port)
        heartbeat.wait_for_cluster(["127.0.0.1", "127.0.0.1"], 0, ports=[a.port, b.port],
                                   start_server=False, poll_s=0.05, timeout_s=10)
    finally:
        a.stop()
        b.stop()
    with pytest.raises(TimeoutError):
        heartbeat.wait_for_cluster(["127.0.0.1"], 0, ports=[a.port], start_server=False,
                                   poll_s=0.05, timeout_s=0.3)


def test_parse_pod_name():
    assert k8s.parse_pod_name("transformer-12") == ("transformer", 12)
    assert k8s.parse_pod_name("my-stateful-set-3") == ("my-stateful-set", 3)
    with pytest.raises(ValueError):
        k8s.parse_pod_name("nodash")


def test_discovery_orders_numerically_and_waits_for_ips():
    """12 pods (the reference sorted names lexicographically: 'x-10' < 'x-2')."""
    calls = {"n": 0}

    def list_pods():
        calls["n"] += 1
        pods = [k8s.PodInfo(f"transformer-{i}", f"10.0.0.{i + 1}") for i in (5, 11, 0, 2, 10, 1, 3, 4, 6, 7, 8, 9)]
        pods.append(k8s.PodInfo("transformer-db-0", "10.9.9.9"))  # other StatefulSet
        pods.append(k8s.PodInfo("unrelated", "10.9.9.8"))
        if calls["n"] < 3:  # pod 7 not scheduled yet
            pods = [p if p.name != "transformer-7" else k8s.PodInfo(p.name, None) for p in pods]
        return pods

    ips = k8s.discover_peers("transformer-3", 12, list_pods, poll_s=0.01, timeout_s=5)
    assert ips == [f"10.0.0.{i + 1}" for i in range(12)]
    assert calls["n"] == 3


def test_discovery_timeout():
    with pytest.raises(TimeoutError):
        k8s.discover_peers("t-0", 3, lambda: [k8s.PodInfo("t-0", "1.1.1.1")], poll_s=0.01, timeout_s=0.1)


def test_bootstrap_k8s_mode(monkeypatch):
    srv = heartbeat.start_heartbeat_server(0)
    port = srv.port
    srv.stop()
    monkeypatch.setenv("THIS_POD_NAME", "tr-1")
    pods = [k8s.PodInfo("tr-0", "127.0.0.1"), k8s.PodInfo("tr-1", "127.0.0.1")]
    spec = rendezvous.bootstrap(2, heartbeat_port=port, master_port=4242, list_pods=lambda: pods,
                                heartbeat_timeout_s=10)
    try:
        assert (spec.node_rank, spec.num_nodes, spec.master_addr, spec.master_port) == (1, 2, "127.0.0.1", 4242)
        saved = dict(os.environ)
        rendezvous.export_env(spec, 8, 3)
        assert os.environ["RANK"] == "11" and os.environ["WORLD_SIZE"] == "16"
        assert os.environ["LOCAL_RANK"] == "3" and os.environ["MASTER_ADDR"] == "127.0.0.1"
    finally:
        os.environ.clear()
        os.environ.update(saved)
        spec.heartbeat.stop()


def test_bootstrap_local_mode(monkeypatch):
    monkeypatch.delenv("THIS_POD_NAME", raising=False)
    spec = rendezvous.bootstrap(3)
    assert spec.chief and spec.num_nodes == 1


def test_launcher_failure_detection():
    """One rank dies -> the others are terminated and its exit code returned."""
    spec = rendezvous.ClusterSpec(0, 1, ["127.0.0.1"], "127.0.0.1", 29999)
    code = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "assert os.environ['WORLD_SIZE'] == '3'\n"
            "time.sleep(0.3) if r == 1 else time.sleep(120)\n"
            "sys.exit(5 if r == 1 else 0)\n")
    t0 = time.time()
    rc = launch.launch(["-c", code], 3, spec, poll_s=0.05)
    assert rc == 5
    assert time.time() - t0 < 60


def test_launcher_success():
    spec = rendezvous.ClusterSpec(0, 1, ["127.0.0.1"], "127.0.0.1", 29999)
    rc = launch.launch(["-c", "import os; assert int(os.environ['LOCAL_RANK']) < 2"], 2, spec, poll_s=0.05)
    assert rc == 0
