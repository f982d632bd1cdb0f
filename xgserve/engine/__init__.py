from .engine import EngineConfig, LLMEngine
from .request import EngineRequest, RequestOutput, RequestType, SamplingParams

__all__ = ["EngineConfig", "LLMEngine", "EngineRequest", "RequestOutput", "RequestType", "SamplingParams"]
