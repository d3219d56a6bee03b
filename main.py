"""V-Gate entry point (drop-in): ``uvicorn main:app`` or ``python main.py``.

The role (gateway / worker), model and everything else come from config.yaml /
``VGATE_*`` environment variables (see vgate/config.py). For tensor-parallel
workers launch one process per GPU with torchrun; TP rank 0 serves HTTP, the
other ranks run the engine follower loop (see vgate/runtime/engine.py).
"""
from __future__ import annotations

import os

from vgate.api.app import ChatCompletionRequest, ChatMessage, create_app, messages_to_prompt  # noqa: F401
from vgate.config import get_config

config = get_config()
IS_WORKER = config.role == "worker"
APP_VERSION = config.version
app = create_app(config)


def main() -> None:
    tp = config.model.tensor_parallel_size
    rank = int(os.environ.get("RANK", "0"))
    if tp > 1 and rank % tp != 0:
        # follower rank: no HTTP server, just the engine lock-step loop
        from vgate.backends.native import NativeBackend
        NativeBackend().load_model(config.model)
        return
    if config.server.http == "uvicorn":
        import uvicorn
        uvicorn.run(app, host=config.server.host, port=config.server.port, log_level="warning",
                    access_log=False, timeout_keep_alive=config.server.timeout_keep_alive,
                    limit_concurrency=config.server.max_connections or None)
        return
    from vgate.api.server import run
    sc = config.server
    run(app, host=sc.host, port=sc.port, timeout_keep_alive=sc.timeout_keep_alive,
        timeout_request=sc.timeout_request, max_connections=sc.max_connections)


if __name__ == "__main__":
    main()
