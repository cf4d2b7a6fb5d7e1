"""jmt — MI355X-native (gfx950) runtime of the Joint-Multimodal-Transformer fusion hot path.

libjmt_hip.so (csrc/, C-ABI in include/jmt.h) holds every kernel; jmt.functional wraps them in
autograd functions; jmt.nn / models.* / losses.* are the drop-in modules."""
from ._lib import load as load_library, JMTError  # noqa: F401
from .functional import compute_mode, set_compute_dtype, compute_dtype  # noqa: F401

__version__ = "0.1.0"
