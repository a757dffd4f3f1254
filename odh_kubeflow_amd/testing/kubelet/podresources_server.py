"""kubelet pod-resources gRPC server stand-in (``v1.PodResourcesLister/List`` on a unix socket).

Test platform only: the production node agent (``nodeagent/podresources.py``) only ever runs
the client.  The wire encoding is the production module's, so the agent's decoder is what the
tests exercise.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

from ...nodeagent.podresources import ContainerDevices, ContainerResources, PodResources, encode_list_response


class FakePodResourcesServer:
    """A kubelet stand-in serving ``v1.PodResourcesLister/List`` on a unix socket (tests and
    the in-process cluster harness)."""

    def __init__(self, socket_path: str):
        self.socket_path = socket_path
        self.pods: Dict[Tuple[str, str], PodResources] = {}
        self._server = None

    def assign(self, namespace: str, name: str, container: str, resource: str, device_ids: List[str]) -> None:
        self.pods[(namespace, name)] = PodResources(name, namespace, [ContainerResources(
            container, [ContainerDevices(resource, list(device_ids))])])

    def release(self, namespace: str, name: str) -> None:
        self.pods.pop((namespace, name), None)

    def start(self) -> "FakePodResourcesServer":
        from concurrent.futures import ThreadPoolExecutor

        import grpc

        def list_handler(_req, _ctx):
            return list(self.pods.values())

        handler = grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
            "List": grpc.unary_unary_rpc_method_handler(list_handler, request_deserializer=lambda b: b,
                                                        response_serializer=encode_list_response)})
        self._server = grpc.server(ThreadPoolExecutor(max_workers=2))
        self._server.add_generic_rpc_handlers((handler,))
        self._server.add_insecure_port(f"unix://{self.socket_path}")
        self._server.start()
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(None)
            self._server = None
