"""Minimal Kubernetes API client (in-cluster service account or kubeconfig
token), enough for the node labeller, the partition manager, the operator and
``mxk8s doctor``: GET / LIST, POST, PUT, DELETE and JSON merge-PATCH over HTTPS
with the cluster CA, plus the REST path of any manifest.  No kubernetes Python
package is needed (none is installed in the image)."""
from __future__ import annotations

import json
import os
import socket
import ssl
import urllib.error
import urllib.parse
import urllib.request
from typing import Optional

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"HTTP {status}: {msg}")
        self.status = status


class KubeClient:
    def __init__(self, server: str, token: Optional[str] = None, ca_file: Optional[str] = None,
                 insecure: bool = False, timeout: float = 10.0):
        self.server = server.rstrip("/")
        self.token = token
        self.timeout = timeout
        if self.server.startswith("https"):
            ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
            if insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            self._ctx = ctx
        else:
            self._ctx = None

    @classmethod
    def in_cluster(cls, sa_dir: str = SA_DIR) -> "KubeClient":
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        with open(os.path.join(sa_dir, "token")) as f:
            token = f.read().strip()
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", token, os.path.join(sa_dir, "ca.crt"))

    def _req(self, method: str, path: str, body=None, content_type="application/json"):
        data = None if body is None else json.dumps(body).encode()
        req = urllib.request.Request(self.server + path, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout, context=self._ctx) as r:
                return json.loads(r.read() or b"{}")
        except urllib.error.HTTPError as e:
            raise KubeError(e.code, e.read().decode(errors="replace")[:500]) from None

    def get(self, path: str) -> dict:
        return self._req("GET", path)

    def merge_patch(self, path: str, patch: dict) -> dict:
        return self._req("PATCH", path, patch, "application/merge-patch+json")

    def get_node(self, name: str) -> dict:
        return self.get(f"/api/v1/nodes/{name}")

    def patch_node_labels(self, name: str, labels: dict) -> dict:
        """labels: value None deletes the label (JSON merge patch)."""
        return self.merge_patch(f"/api/v1/nodes/{name}", {"metadata": {"labels": labels}})

    def list(self, path: str, label_selector: Optional[str] = None) -> list:
        return self.list_with_version(path, label_selector)[0]

    def list_with_version(self, path: str, label_selector: Optional[str] = None) -> tuple[list, str]:
        """(items, the collection's resourceVersion): where a watch resumes."""
        q = "?labelSelector=" + urllib.parse.quote(label_selector) if label_selector else ""
        doc = self._req("GET", path + q)
        return doc.get("items", []), str(doc.get("metadata", {}).get("resourceVersion", ""))

    def watch(self, path: str, resource_version: str = "", timeout_s: float = 30.0,
              label_selector: Optional[str] = None, on_open=None):
        """Yield the watch events ({"type": ADDED|MODIFIED|DELETED|ERROR,
        "object": ...}) of a collection after ``resource_version``, until the
        server ends the watch (``timeoutSeconds``).  ``on_open(cancel)`` gets a
        callable that ends this watch from another thread (it shuts the
        long-poll connection down, so the blocked read returns at once)."""
        q = {"watch": "1", "timeoutSeconds": str(max(1, int(timeout_s)))}
        if resource_version:
            q["resourceVersion"] = resource_version
        if label_selector:
            q["labelSelector"] = label_selector
        req = urllib.request.Request(self.server + path + "?" + urllib.parse.urlencode(q))
        req.add_header("Accept", "application/json")
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        cancelled = []

        def cancel(r):
            cancelled.append(True)
            _shutdown(r)

        try:
            with urllib.request.urlopen(req, timeout=timeout_s + 10, context=self._ctx) as r:
                if on_open is not None:
                    on_open(lambda: cancel(r))
                for line in r:
                    line = line.strip()
                    if line:
                        yield json.loads(line)
        except urllib.error.HTTPError as e:
            raise KubeError(e.code, e.read().decode(errors="replace")[:500]) from None
        except (OSError, ValueError, AttributeError):
            if not cancelled:
                raise
            return      # cancelled by the caller (connection shut down under the read)

    def create(self, collection: str, obj: dict) -> dict:
        return self._req("POST", collection, obj)

    def replace(self, path: str, obj: dict) -> dict:
        return self._req("PUT", path, obj)

    def delete(self, path: str, propagation: Optional[str] = None) -> dict:
        """``propagation``: Background | Foreground | Orphan (DeleteOptions).
        The API server's default for batch/v1 Jobs is Orphan: the Job's pods
        keep running and the Job lingers behind the orphan finalizer."""
        body = None if propagation is None else {"kind": "DeleteOptions", "apiVersion": "v1",
                                                 "propagationPolicy": propagation}
        return self._req("DELETE", path, body)

    def patch_status(self, path: str, status: dict) -> dict:
        return self.merge_patch(path + "/status", {"status": status})


# kinds whose objects are not namespaced (the ones this stack manages)
CLUSTER_SCOPED = {"Namespace", "Node", "ClusterRole", "ClusterRoleBinding",
                  "CustomResourceDefinition", "GPUStackPolicy", "RuntimeClass", "PriorityClass"}
_PLURALS = {"GPUStackPolicy": "gpustackpolicies", "PriorityClass": "priorityclasses"}


def plural(kind: str) -> str:
    return _PLURALS.get(kind, kind.lower() + ("es" if kind.endswith("s") else "s"))


def collection_path(api_version: str, kind: str, namespace: Optional[str] = None) -> str:
    """REST collection path of ``kind`` (namespaced kinds need ``namespace``)."""
    base = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
    if kind in CLUSTER_SCOPED or not namespace:
        return f"{base}/{plural(kind)}"
    return f"{base}/namespaces/{namespace}/{plural(kind)}"


def object_path(obj: dict, default_namespace: Optional[str] = None) -> str:
    md = obj.get("metadata", {})
    ns = None if obj["kind"] in CLUSTER_SCOPED else (md.get("namespace") or default_namespace)
    return collection_path(obj["apiVersion"], obj["kind"], ns) + "/" + md["name"]


def _shutdown(resp) -> None:
    """Unblock a thread reading a streaming HTTP response and close it."""
    try:
        sock = resp.fp.raw._sock            # http.client.HTTPResponse over a socket
        sock.shutdown(socket.SHUT_RDWR)
    except (AttributeError, OSError):
        pass
    try:
        resp.close()
    except Exception:                       # already closed / mid-read in the other thread
        pass
