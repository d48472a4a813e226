"""gin.config: the binding tables the reference imports (`from gin.config import _CONFIG,
_OPERATIVE_CONFIG`, src/model.py:10, src/callbacks.py:22, src/utils.py:8-9)."""
from greedy_multimodal_learning_amd.gin_lite import _CONFIG, _REGISTRY, parse_config  # noqa: F401

_OPERATIVE_CONFIG = {}
