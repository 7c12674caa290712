"""hipserve — MI355X-native LLM serving engine for the llms-on-kubernetes stack.

Layers: ``server`` (OpenAI HTTP API) -> ``engine`` (scheduler, paged KV pool,
model runner, hipGraph decode) -> ``models`` (Llama / Mixtral) -> ``ops``
(gfx950 HIP kernels in ``_C.so``) and ``parallel`` (RCCL tensor parallel).
``gateway`` holds the model-name router and the ingress emulator; ``weights``
the safetensors / GGUF / dummy loaders.
"""
__version__ = "0.1.0"
