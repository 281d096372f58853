"""A fake kubelet for contract tests and offline drills.

Serves ``v1beta1.Registration/Register`` on ``<dir>/kubelet.sock`` like the
kubelet's device manager, records every RegisterRequest, and then acts as
the kubelet's client of the registered plugin: ListAndWatch, Allocate,
GetPreferredAllocation, GetDevicePluginOptions, PreStartContainer.
``restart()`` simulates a kubelet restart (the kubelet removes every socket
in the plugin directory and re-creates kubelet.sock).
"""
from __future__ import annotations

import concurrent.futures
import os
import queue
import threading
from typing import Optional

import grpc

from . import api


class FakeKubelet:
    def __init__(self, plugin_dir: str):
        self.plugin_dir = plugin_dir
        self.socket = os.path.join(plugin_dir, api.KUBELET_SOCKET_NAME)
        self.registrations: "queue.Queue" = queue.Queue()
        self.all_registrations: list = []
        self._server: Optional[grpc.Server] = None
        self._lock = threading.Lock()

    # Registration service
    def Register(self, request, context):
        if request.version != api.API_VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"bad version {request.version}")
        with self._lock:
            self.all_registrations.append(request)
        self.registrations.put(request)
        return api.Empty()

    def start(self) -> "FakeKubelet":
        os.makedirs(self.plugin_dir, exist_ok=True)
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        srv = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=4))
        srv.add_generic_rpc_handlers((api.generic_handler("Registration", self),))
        srv.add_insecure_port("unix:" + self.socket)
        srv.start()
        self._server = srv
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=0.2).wait()
            self._server = None

    def restart(self) -> None:
        """Kubelet restart: stop, wipe every socket in the plugin dir, start."""
        self.stop()
        for name in os.listdir(self.plugin_dir):
            p = os.path.join(self.plugin_dir, name)
            if name.endswith(".sock"):
                try:
                    os.unlink(p)
                except FileNotFoundError:
                    pass
        self.start()

    def wait_registration(self, timeout: float = 10.0):
        return self.registrations.get(timeout=timeout)

    # kubelet -> plugin client
    def plugin_channel(self, endpoint: str) -> grpc.Channel:
        ch = grpc.insecure_channel("unix:" + os.path.join(self.plugin_dir, endpoint))
        grpc.channel_ready_future(ch).result(timeout=10)
        return ch

    def plugin_stub(self, endpoint: str):
        return api.Stub(self.plugin_channel(endpoint), "DevicePlugin")
