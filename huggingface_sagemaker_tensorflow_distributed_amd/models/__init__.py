from .bert import RobertaForMaskedLM, TransformerForSequenceClassification, build_model
from .config import REGISTRY, ModelConfig, resolve_config
from .hf_io import from_pretrained, hf_state_dict, load_hf_state_dict, save_pretrained

__all__ = [
    "ModelConfig", "REGISTRY", "resolve_config", "build_model", "TransformerForSequenceClassification",
    "RobertaForMaskedLM", "from_pretrained", "save_pretrained", "hf_state_dict", "load_hf_state_dict",
]
