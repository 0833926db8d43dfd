"""HTTP heartbeat: a liveness endpoint plus a start-up rendezvous barrier.

Reference: distributed_training_transformer/cluster/heartbeat.py:13-69 — every
pod serves "Server operational" on a port and polls every peer (itself
included) until all answer. Kept as the liveness endpoint of the pods; the
barrier gains a timeout and a stop handle (the reference could wait forever).
"""
from __future__ import annotations

import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Iterable, Optional
from urllib.error import URLError
from urllib.request import urlopen

HEARTBEAT_MESSAGE = "Server operational"


class _Handler(BaseHTTPRequestHandler):
    def do_GET(self):  # noqa: N802
        body = HEARTBEAT_MESSAGE.encode("utf-8")
        self.send_response(200)
        self.send_header("Content-type", "text/plain; charset=utf-8")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *args):  # silence
        pass


class HeartbeatServer:
    def __init__(self, port: int, host: str = ""):
        self.httpd = ThreadingHTTPServer((host, port), _Handler)
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="liveness_server",
                                       daemon=True)
        self.thread.start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def start_heartbeat_server(port: int) -> HeartbeatServer:
    return HeartbeatServer(port)


def probe(host: str, port: int, timeout: float = 2.0) -> bool:
    try:
        with urlopen(f"http://{host}:{port}", timeout=timeout) as c:
            msg = c.read().decode("utf-8")
    except (URLError, OSError):
        return False
    if msg != HEARTBEAT_MESSAGE:
        raise RuntimeError(f"Unexpected response from peer heartbeat server:\n{msg}")
    return True


def wait_for_cluster(hosts: Iterable[str], port: int, verbose: bool = False,
                     poll_s: float = 2.0, timeout_s: Optional[float] = None,
                     start_server: bool = True, ports: Optional[Iterable[int]] = None) -> Optional[HeartbeatServer]:
    """Start our heartbeat server, then block until every host answers."""
    srv = None
    if start_server:
        if verbose:
            print("Starting heartbeat server.")
        srv = start_heartbeat_server(port)
    if verbose:
        print("Trying to connect to peers.")
    deadline = None if timeout_s is None else time.time() + timeout_s
    hosts = list(hosts)
    plist = list(ports) if ports is not None else [port] * len(hosts)
    for host, p in zip(hosts, plist):
        while not probe(host, p):
            if deadline is not None and time.time() > deadline:
                raise TimeoutError(f"heartbeat: peer {host}:{p} unreachable")
            time.sleep(poll_s)
    if verbose:
        print("All peers reachable.")
    return srv
