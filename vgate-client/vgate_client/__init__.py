"""V-Gate Python client SDK (sync + async), drop-in with the reference ``vgate-client`` 0.1.0.

    from vgate_client import VGate, AsyncVGate
    client = VGate(base_url="http://localhost:8000", api_key="sk-...")
    resp = client.chat.create(model="Qwen/Qwen2.5-1.5B-Instruct", messages=[{"role": "user", "content": "Hi"}])
    for chunk in client.chat.stream(model="...", messages=[...]):
        print(chunk.choices[0].delta.content or "", end="")
"""
from .client import AsyncChatStream, AsyncVGate, SyncChatStream, VGate
from .exceptions import AuthenticationError, ConnectionError, RateLimitError, ServerError, VGateError
from .models import (ChatCompletion, ChatCompletionChunk, ChatCompletionChunkChoice, ChatCompletionDelta,
                     ChatMessage, Choice, EmbeddingData, EmbeddingResponse, HealthResponse, RateLimitInfo,
                     ResponseMessage, Usage)

__version__ = "0.1.0"
__all__ = [
    "VGate", "AsyncVGate", "SyncChatStream", "AsyncChatStream",
    "ChatCompletion", "ChatCompletionChunk", "ChatCompletionChunkChoice", "ChatCompletionDelta", "Choice",
    "ResponseMessage", "EmbeddingResponse", "EmbeddingData", "HealthResponse", "Usage", "RateLimitInfo",
    "ChatMessage", "VGateError", "AuthenticationError", "RateLimitError", "ServerError", "ConnectionError",
]
