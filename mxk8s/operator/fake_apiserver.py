"""In-process fake Kubernetes API server for the operator's contract tests
(the same role ``deviceplugin/fake_kubelet.py`` plays for the plugin).

Stores objects by REST path and implements what the controller uses: GET
(object or collection, ``labelSelector`` equality terms, the collection's
``metadata.resourceVersion``), watches (``?watch=1&resourceVersion=&
timeoutSeconds=``: newline-delimited events after that version), POST (409 on
an existing name, also while a deleted object still has finalizers), PUT
(replace, bumps ``metadata.generation`` when ``spec`` changes), JSON
merge-PATCH (also on ``/status``), DELETE with DeleteOptions.  Every write
bumps ``metadata.resourceVersion``.  ``objects`` is directly inspectable and
mutable by tests (to simulate drift or a DaemonSet becoming ready).

Real-server behaviours a controller must survive, modelled here:

* ``job_orphan_linger`` (s): DELETE of a batch/v1 Job without a propagation
  policy defaults to Orphan — the Job stays, with ``deletionTimestamp`` and
  the ``orphan`` finalizer, until the garbage collector releases it; a POST
  of the same name meanwhile gets 409 AlreadyExists;
* ``normalize``: the server stores resource quantities in canonical form
  (``0.5`` -> ``500m``, ``1024Mi`` -> ``1Gi``), defaults container fields and
  lets a "mutating webhook" inject a volume and an env var (named list items
  the rendered object does not have, at the front of the list).
"""
from __future__ import annotations

import copy
import http.server
import itertools
import json
import threading
import time
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


def canonical_quantity(v):
    """Kubernetes' canonical spelling of a quantity (decimal: milli-units below
    one, integers otherwise; binary: the largest exact Ki..Ei suffix)."""
    from . import parse_quantity
    q = parse_quantity(v)
    if q is None:
        return v
    if isinstance(v, str) and v.endswith("i"):
        for suf, mul in (("Ei", 2 ** 60), ("Pi", 2 ** 50), ("Ti", 2 ** 40), ("Gi", 2 ** 30),
                         ("Mi", 2 ** 20), ("Ki", 2 ** 10)):
            if q % mul == 0:
                return f"{q // mul}{suf}"
    if q.denominator == 1:
        return str(q.numerator)
    milli = q * 1000
    return f"{int(milli)}m" if milli.denominator == 1 else str(float(q))


def _normalize(obj: dict) -> None:
    def walk(o, key=None):
        if isinstance(o, dict):
            for k, v in list(o.items()):
                if key in ("requests", "limits") and isinstance(v, (str, int, float)):
                    o[k] = canonical_quantity(v)
                else:
                    walk(v, k)
        elif isinstance(o, list):
            for x in o:
                walk(x, key)
    walk(obj)
    pod = obj.get("spec", {}).get("template", {}).get("spec")
    if not isinstance(pod, dict):
        return
    vols = pod.setdefault("volumes", [])
    if not any(v.get("name") == "kube-api-access" for v in vols):
        vols.insert(0, {"name": "kube-api-access", "projected": {"sources": []}})
    for c in pod.get("containers", []) + pod.get("initContainers", []):
        c.setdefault("terminationMessagePath", "/dev/termination-log")
        env = c.setdefault("env", [])
        if not any(e.get("name") == "INJECTED_BY_WEBHOOK" for e in env):
            env.insert(0, {"name": "INJECTED_BY_WEBHOOK", "value": "1"})
        for p in c.get("ports", []):
            p.setdefault("protocol", "TCP")


class FakeApiServer:
    def __init__(self, normalize: bool = False, job_orphan_linger: float = 0.0):
        self.objects: dict[str, dict] = {}
        self.lock = threading.Condition()
        self.requests: list[tuple[str, str]] = []
        self.events: list[tuple[int, str, str, dict]] = []   # (rv, type, path, object)
        self._rv = itertools.count(1)
        self._last_rv = 0
        self._httpd = None
        self.normalize = normalize
        self.job_orphan_linger = job_orphan_linger
        self._lingering: list[tuple[threading.Timer, object]] = []

    # ------------------------------------------------------------ storage
    def _bump(self, obj: dict) -> None:
        self._last_rv = next(self._rv)
        obj.setdefault("metadata", {})["resourceVersion"] = str(self._last_rv)

    def _event(self, etype: str, path: str, obj: dict) -> None:
        self.events.append((self._last_rv, etype, path, copy.deepcopy(obj)))
        self.lock.notify_all()

    def put_object(self, path: str, obj: dict) -> None:
        with self.lock:
            o = copy.deepcopy(obj)
            o.setdefault("metadata", {}).setdefault("uid", str(uuid.uuid4()))
            o["metadata"].setdefault("generation", 1)
            etype = "MODIFIED" if path in self.objects else "ADDED"
            self._bump(o)
            self.objects[path] = o
            self._event(etype, path, o)

    def _release_later(self, path: str, uid: str) -> None:
        def release():
            with self.lock:
                cur = self.objects.get(path)
                if cur is not None and cur["metadata"].get("uid") == uid:
                    del self.objects[path]
                    self._bump({})
                    self._event("DELETED", path, cur)
        t = threading.Timer(self.job_orphan_linger, release)
        t.daemon = True
        self._lingering.append((t, release))
        t.start()

    def release_lingering(self) -> None:
        """The garbage collector's release of every lingering Job, now (tests
        drive it instead of sleeping past ``job_orphan_linger``, which a
        loaded machine can overshoot before the assertion that needs the Job
        still there)."""
        pending, self._lingering = self._lingering, []
        for t, release in pending:
            t.cancel()
            release()

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
                    return 200, {"kind": "List", "metadata": {"resourceVersion": str(self._last_rv)},
                                 "items": items}
                return 404, {"reason": "NotFound", "message": f"{opath} not found"}
            if method == "POST":
                name = body.get("metadata", {}).get("name")
                p = f"{opath}/{name}"
                if p in self.objects:
                    return 409, {"reason": "AlreadyExists", "message": p}
                o = copy.deepcopy(body)
                o["metadata"].update(uid=str(uuid.uuid4()), generation=1)
                if self.normalize:
                    _normalize(o)
                self._bump(o)
                self.objects[p] = o
                self._event("ADDED", p, o)
                return 201, copy.deepcopy(o)
            if opath not in self.objects:
                return 404, {"reason": "NotFound", "message": f"{opath} not found"}
            cur = self.objects[opath]
            if method == "DELETE":
                policy = (body or {}).get("propagationPolicy")
                if (cur.get("kind") == "Job" or "/jobs/" in opath) and policy in (None, "Orphan") \
                        and self.job_orphan_linger > 0:
                    if "deletionTimestamp" not in cur["metadata"]:
                        cur["metadata"]["deletionTimestamp"] = time.strftime("%Y-%m-%dT%H:%M:%SZ")
                        cur["metadata"]["finalizers"] = ["orphan"]
                        self._bump(cur)
                        self._event("MODIFIED", opath, cur)
                        self._release_later(opath, cur["metadata"]["uid"])
                    return 200, copy.deepcopy(cur)
                del self.objects[opath]
                self._bump({})
                self._event("DELETED", opath, cur)
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
                    if self.normalize:
                        _normalize(o)
                    self.objects[opath] = cur = o
                self._bump(cur)
                self._event("MODIFIED", opath, cur)
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
                self._event("MODIFIED", opath, cur)
                return 200, copy.deepcopy(cur)
        return 405, {"message": method}

    def watch_stream(self, raw_path: str):
        """Events of one collection after ?resourceVersion=, until timeoutSeconds."""
        url = urllib.parse.urlparse(raw_path)
        coll = url.path.rstrip("/")
        q = urllib.parse.parse_qs(url.query)
        since = int((q.get("resourceVersion") or ["0"])[0] or 0)
        sel = q.get("labelSelector", [""])[0]
        end = time.monotonic() + float((q.get("timeoutSeconds") or ["30"])[0])
        sent = since
        while True:
            with self.lock:
                batch = [(rv, t, o) for rv, t, p, o in self.events
                         if rv > sent and p.rsplit("/", 1)[0] == coll and _match(o, sel)]
                if not batch:
                    left = end - time.monotonic()
                    if left <= 0:
                        return
                    self.lock.wait(min(left, 0.2))
                    continue
            for rv, t, o in batch:
                sent = max(sent, rv)
                yield {"type": t, "object": o}

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
                q = urllib.parse.parse_qs(urllib.parse.urlparse(self.path).query)
                if self.command == "GET" and (q.get("watch") or [""])[0] in ("1", "true"):
                    srv.requests.append(("WATCH", urllib.parse.urlparse(self.path).path))
                    self.send_response(200)
                    self.send_header("Content-Type", "application/json")
                    self.end_headers()      # HTTP/1.0: the stream ends when we close
                    try:
                        for ev in srv.watch_stream(self.path):
                            self.wfile.write((json.dumps(ev) + "\n").encode())
                            self.wfile.flush()
                    except (BrokenPipeError, ConnectionResetError):
                        pass
                    return
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
        self._httpd.daemon_threads = True
        threading.Thread(target=self._httpd.serve_forever, daemon=True).start()
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self._httpd.server_address[1]}"

    def stop(self) -> None:
        for t, _ in self._lingering:
            t.cancel()
        self._lingering = []
        if self._httpd:
            self._httpd.shutdown()
            self._httpd.server_close()

    def count(self, method: str) -> int:
        return sum(1 for m, _ in self.requests if m == method)


__all__ = ["FakeApiServer", "canonical_quantity", "merge"]
