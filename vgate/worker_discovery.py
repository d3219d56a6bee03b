"""DNS-based worker membership (headless Service -> stable per-pod endpoints).

Semantics (reference ``vgate/worker_discovery.py``):
* forward-resolve the Service name (``getaddrinfo(AF_UNSPEC)``), then
  reverse-resolve every address to the pod's stable DNS name so metric labels
  survive pod restarts; fall back to the address (logged once per address);
* ``EAI_NONAME`` / ``EAI_NODATA`` are an authoritative EMPTY answer; every other
  resolver failure raises :class:`TransientResolutionError` so callers keep the
  members they have (a DNS outage must never empty a healthy pool);
* IPv6 literals are bracketed in URLs; a PTR equal to the Service name itself is
  not an identity; resolvers are injectable for tests.
"""
from __future__ import annotations

import ipaddress
import socket
from typing import Callable, List, Optional, Sequence, Tuple

from vgate.logging_config import get_logger

logger = get_logger("vgate.discovery")

AUTHORITATIVE_EMPTY = {getattr(socket, n) for n in ("EAI_NONAME", "EAI_NODATA") if hasattr(socket, n)}


class TransientResolutionError(RuntimeError):
    """The resolver could not answer (distinct from answering 'no records')."""


ForwardResolver = Callable[[str, int], Sequence[str]]
ReverseResolver = Callable[[str], str]


def default_forward(host: str, port: int) -> Sequence[str]:
    infos = socket.getaddrinfo(host, port, socket.AF_UNSPEC, socket.SOCK_STREAM)
    return sorted({i[4][0] for i in infos})


def default_reverse(address: str) -> str:
    return socket.gethostbyaddr(address)[0]


def host_for_url(host: str) -> str:
    if host.startswith("["):
        return host
    try:
        if ipaddress.ip_address(host).version == 6:
            return f"[{host}]"
    except ValueError:
        pass
    return host


class DnsWorkerDiscovery:
    def __init__(self, dns_name: str, port: int = 8000, scheme: str = "http",
                 forward_resolver: Optional[ForwardResolver] = None,
                 reverse_resolver: Optional[ReverseResolver] = None):
        self.dns_name = dns_name
        self.port = port
        self.scheme = scheme
        self._forward = forward_resolver or default_forward
        self._reverse = reverse_resolver or default_reverse
        self._logged_fallbacks: set = set()

    def resolve(self) -> List[str]:
        try:
            addrs = self._forward(self.dns_name, self.port)
        except socket.gaierror as e:
            if e.errno not in AUTHORITATIVE_EMPTY:
                raise TransientResolutionError(f"resolver could not answer for {self.dns_name!r}: {e}") from e
            logger.debug("Worker DNS name has no records", extra={"extra_data": {"dns_name": self.dns_name}})
            return []
        except OSError as e:
            raise TransientResolutionError(f"resolver failure for {self.dns_name!r}: {e}") from e
        return sorted({self._endpoint(a) for a in addrs})

    def _endpoint(self, address: str) -> str:
        host, stable = self._stable_name(address)
        if not stable and address not in self._logged_fallbacks:
            self._logged_fallbacks.add(address)
            logger.warning("Reverse lookup failed; using the pod address as its identity. "
                           "Metric labels will churn as pods restart.",
                           extra={"extra_data": {"address": address, "dns_name": self.dns_name}})
        return f"{self.scheme}://{host_for_url(host)}:{self.port}"

    def _stable_name(self, address: str) -> Tuple[str, bool]:
        try:
            name = self._reverse(address)
        except (socket.herror, socket.gaierror, OSError):
            return address, False
        if not name or name.rstrip(".") == self.dns_name.rstrip("."):
            return address, False
        return name.rstrip("."), True
