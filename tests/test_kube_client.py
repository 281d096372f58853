"""KubeClient error paths (a connection error must surface as the
real OSError / URLError, and a cancelled watch must end quietly)."""
import socket
import threading
import urllib.error
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from mxk8s.utils.kube import KubeClient


def _closed_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("call", ["get", "create", "replace", "delete", "patch"])
def test_connection_refused_raises_oserror_not_nameerror(call):
    c = KubeClient(f"http://127.0.0.1:{_closed_port()}", timeout=2.0)
    with pytest.raises((urllib.error.URLError, OSError)) as ei:
        if call == "get":
            c.get("/api/v1/nodes")
        elif call == "create":
            c.create("/api/v1/namespaces", {"metadata": {"name": "x"}})
        elif call == "replace":
            c.replace("/api/v1/namespaces/x", {"metadata": {"name": "x"}})
        elif call == "delete":
            c.delete("/api/v1/namespaces/x")
        else:
            c.merge_patch("/api/v1/nodes/n", {"metadata": {}})
    assert not isinstance(ei.value, NameError)


class _Stream(BaseHTTPRequestHandler):
    """A watch that sends one event and then holds the connection open."""

    def do_GET(self):
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.end_headers()
        self.wfile.write(b'{"type": "ADDED", "object": {"metadata": {"name": "a"}}}\n')
        self.wfile.flush()
        self.server.hold.wait(10)

    def log_message(self, *a):
        pass


def test_cancelled_watch_ends_quietly():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Stream)
    srv.hold = threading.Event()
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        c = KubeClient(f"http://127.0.0.1:{srv.server_address[1]}")
        cancel = []
        events = []
        for ev in c.watch("/api/v1/pods", timeout_s=5, on_open=cancel.append):
            events.append(ev)
            cancel[0]()          # shut the long poll down from "another thread"
        assert [e["type"] for e in events] == ["ADDED"]
    finally:
        srv.hold.set()
        srv.shutdown()
        srv.server_close()
