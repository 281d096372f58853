"""In-process fake Kubernetes API server for the operator's contract tests
(the same role ``deviceplugin/fake_kubelet.py`` plays for the plugin).

Stores objects by REST path and implements what the controller uses: GET
(object or collection, ``labelSelector`` equality terms), POST (409 on an
existing name), PUT (replace, bumps ``metadata.generation`` when ``spec``
changes), JSON merge-PATCH (also on ``/status``), DELETE.  Every write bumps
``metadata.resourceVersion``.  ``objects`` is directly inspectable and
mutable by tests (to simulate drift or a DaemonSet becoming ready).
"""
from __future__ import annotations

import copy
import http.server
import itertools
import json
import threading
import urllib.parse
import uuid


def merge(dst: dict, patch: dict) -> dict:
    """RFC 7386 JSON merge patch."""
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _match(obj: dict, selector: str) -> bool:
    labels = obj.get("metadata", {}).get("labels", {}) or {}
    for term in filter(None, selector.split(",")):
        k, _, v = term.partition("=")
        if labels.get(k) != v:
            return False
    return True


class FakeApiServer:
    def __init__(self):
        self.objects: dict[str, dict] = {}
        self.lock = threading.Lock()
        self.requests: list[tuple[str, str]] = []
        self._rv = itertools.count(1)
        self._httpd = None

    # ------------------------------------------------------------ storage
    def _bump(self, obj: dict) -> None:
        obj.setdefault("metadata", {})["resourceVersion"] = str(next(self._rv))

    def put_object(self, path: str, obj: dict) -> None:
        with self.lock:
            o = copy.deepcopy(obj)
            o.setdefault("metadata", {}).setdefault("uid", str(uuid.uuid4()))
            o["metadata"].setdefault("generation", 1)
            self._bump(o)
            self.objects[path] = o

    def handle(self, method: str, raw_path: str, body: dict | None) -> tuple[int, dict]:
        url = urllib.parse.urlparse(raw_path)
        path = url.path.rstrip("/")
        q = urllib.parse.parse_qs(url.query)
        self.requests.append((method, path))
        status_sub = path.endswith("/status")
        opath = path[: -len("/status")] if status_sub else path
        with self.lock:
            if method == "GET":
                if opath in self.objects:
                    return 200, copy.deepcopy(self.objects[opath])
                sel = q.get("labelSelector", [""])[0]
                items = [copy.deepcopy(o) for p, o in sorted(self.objects.items())
                         if p.rsplit("/", 1)[0] == opath and _match(o, sel)]
                if items or self._is_collection(opath):
                    return 200, {"kind": "List", "items": items}
                return 404, {"reason": "NotFound", "message": f"{opath} not found"}
            if method == "POST":
                name = body.get("metadata", {}).get("name")
                p = f"{opath}/{name}"
                if p in self.objects:
                    return 409, {"reason": "AlreadyExists", "message": p}
                o = copy.deepcopy(body)
                o["metadata"].update(uid=str(uuid.uuid4()), generation=1)
                self._bump(o)
                self.objects[p] = o
                return 201, copy.deepcopy(o)
            if opath not in self.objects:
                return 404, {"reason": "NotFound", "message": f"{opath} not found"}
            cur = self.objects[opath]
            if method == "DELETE":
                del self.objects[opath]
                return 200, {"status": "Success"}
            if method == "PUT":
                o = copy.deepcopy(body)
                if status_sub:
                    cur["status"] = o.get("status", {})
                else:
                    o["metadata"]["uid"] = cur["metadata"]["uid"]
                    gen = cur["metadata"].get("generation", 1)
                    o["metadata"]["generation"] = gen + (o.get("spec") != cur.get("spec"))
                    o.setdefault("status", cur.get("status", {}))
                    self.objects[opath] = cur = o
                self._bump(cur)
                return 200, copy.deepcopy(cur)
            if method == "PATCH":
                if status_sub:
                    merge(cur.setdefault("status", {}), (body or {}).get("status", {}))
                else:
                    old_spec = copy.deepcopy(cur.get("spec"))
                    merge(cur, {k: v for k, v in (body or {}).items() if k != "status"})
                    if cur.get("spec") != old_spec:
                        cur["metadata"]["generation"] = cur["metadata"].get("generation", 1) + 1
                self._bump(cur)
                return 200, copy.deepcopy(cur)
        return 405, {"message": method}

    @staticmethod
    def _is_collection(path: str) -> bool:
        """/api/v1/<plural>, /api/v1/namespaces/<ns>/<plural>, /apis/<g>/<v>/<plural>,
        /apis/<g>/<v>/namespaces/<ns>/<plural>."""
        seg = [x for x in path.split("/") if x]
        if not seg:
            return False
        rest = seg[2:] if seg[0] == "api" else seg[3:]
        if rest[:1] == ["namespaces"] and len(rest) >= 2:
            rest = rest[2:]
        return len(rest) == 1

    # --------------------------------------------------------------- HTTP
    def start(self) -> "FakeApiServer":
        srv = self

        class H(http.server.BaseHTTPRequestHandler):
            def _do(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n)) if n else None
                code, out = srv.handle(self.command, self.path, body)
                data = json.dumps(out).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            do_GET = do_POST = do_PUT = do_PATCH = do_DELETE = _do

            def log_message(self, *a):
                pass

        self._httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self._httpd.serve_forever, daemon=True).start()
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self._httpd.server_address[1]}"

    def stop(self) -> None:
        if self._httpd:
            self._httpd.shutdown()
            self._httpd.server_close()
