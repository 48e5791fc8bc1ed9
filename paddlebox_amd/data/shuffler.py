"""Data-shuffle message service (``boxps::PaddleShuffler`` contract,
``box_wrapper.h:672-673``, ``data_set.cc:1906-1935,2440-2604``).

One native ``MsgService`` per process (the reference keeps one in
``BoxWrapper::data_shuffle_``): a TCP full mesh between the ranks with a
sender thread per outbound peer and a receiver thread per inbound peer
(``csrc/host/msg_service.{h,cc}``).  Consumers register a handler and get a
service id; ``send_message(service_id << 16 | rank, ...)`` streams a message
to a peer and the optional callback fires once the peer has handled it;
``wait_done(service_id)`` waits for all of a service's messages.

The ranks' endpoints are exchanged through the ``torch.distributed`` store
(the rendezvous every process already has), so no extra configuration is
needed.  Single-node jobs bind the loopback interface; multi-node jobs bind
all interfaces and publish ``PBX_SHUFFLE_HOST`` (default: this host's
address).
"""
from __future__ import annotations

import os
import socket
import threading
from typing import Callable, Optional

import torch.distributed as dist

from .. import _native

_lock = threading.Lock()
_instance: Optional["PaddleShuffler"] = None


class PaddleShuffler:
    def __init__(self, rank: int, world: int, store=None, tag: str = "pbx_shuffle"):
        self.rank, self.world = int(rank), int(world)
        self.svc = _native.host().MsgService(self.rank, self.world)
        if self.world == 1:
            self.svc.connect(["127.0.0.1:0"])
            return
        single_node = int(os.environ.get("LOCAL_WORLD_SIZE", self.world)) == self.world
        host = os.environ.get("PBX_SHUFFLE_HOST") or ("127.0.0.1" if single_node else _host_addr())
        port = self.svc.listen("127.0.0.1" if single_node else "0.0.0.0", 0)
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        store.set(f"{tag}/{self.rank}", f"{host}:{port}")
        eps = [store.get(f"{tag}/{r}").decode() for r in range(self.world)]
        self.svc.connect(eps)

    # -- boxps::PaddleShuffler API -----------------------------------------
    def register_handler(self, on_receive: Callable[[int, bytes], None]) -> int:
        return self.svc.register_handler(on_receive)

    def unregister_consumer(self, service_id: int):
        self.svc.unregister_consumer(service_id)

    def send_message_callback(self, client_id: int, data: bytes, callback: Optional[Callable[[], None]] = None):
        self.svc.send_message(client_id, data, callback)

    def wait_done(self, service_id: int):
        self.svc.wait_done(service_id)

    def destory(self):  # the reference's spelling
        self.svc.destroy()

    destroy = destory


def _host_addr() -> str:
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return "127.0.0.1"


def get_shuffler(rank: int, world: int) -> PaddleShuffler:
    """Process-wide service (created on first use by the first dataset that
    shuffles globally; every rank creates it at the same point)."""
    global _instance
    with _lock:
        if _instance is None or (_instance.rank, _instance.world) != (rank, world):
            if _instance is not None:
                _instance.destroy()
            _instance = PaddleShuffler(rank, world)
        return _instance


def finalize():
    global _instance
    with _lock:
        if _instance is not None:
            _instance.destroy()
            _instance = None
