"""`import gin` for the reference's train.py / eval.py / src/*.py when the real gin-config
package is absent (it is not installed in this image): the subset the reference uses -
`gin.configurable`, `gin.parse_config_files_and_bindings`, `gin.config._CONFIG` /
`_OPERATIVE_CONFIG` - backed by greedy_multimodal_learning_amd.gin_lite, so a config
bound here also binds the MI355X drop-in classes.  Put `compat/` on PYTHONPATH only
when gin itself is missing."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from greedy_multimodal_learning_amd.gin_lite import (clear_config, config_str, configurable,  # noqa: E402,F401
                                                     parse_config_files_and_bindings, query)
from . import config  # noqa: E402,F401

operative_config_str = config_str
REQUIRED = object()
