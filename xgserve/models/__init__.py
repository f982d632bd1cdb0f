from .config import ModelConfig, get_config, list_models, from_hf_config
from .base import AttnMeta
from .llama import LlamaForCausalLM
from .gpt2 import GPT2ForCausalLM
from .loader import build_model, load_checkpoint, save_checkpoint

__all__ = ["ModelConfig", "get_config", "list_models", "from_hf_config", "AttnMeta", "LlamaForCausalLM",
           "GPT2ForCausalLM", "build_model", "load_checkpoint", "save_checkpoint"]
