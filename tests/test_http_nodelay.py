"""The multi-worker HTTP tier's listening socket (parallel/workers.bind_reuseport) must give accepted
connections TCP_NODELAY.  asyncio only sets it when the socket's proto is IPPROTO_TCP; without it
uvicorn's two writes per response (head, then body) wait for the client's delayed ACK and every
request gains ~40 ms (profiles/r3/README.md)."""
import asyncio
import socket

from ai_agent_kubectl_amd.parallel.workers import bind_reuseport


def test_accepted_connections_have_nodelay():
    s = bind_reuseport("127.0.0.1", 0)
    port = s.getsockname()[1]
    assert s.proto == socket.IPPROTO_TCP
    seen = []

    async def main():
        async def on_conn(reader, writer):
            seen.append(writer.get_extra_info("socket").getsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY))
            writer.close()

        server = await asyncio.start_server(on_conn, sock=s)
        r, w = await asyncio.open_connection("127.0.0.1", port)
        await r.read()
        w.close()
        server.close()
        await server.wait_closed()

    asyncio.run(main())
    assert seen and seen[0] != 0
