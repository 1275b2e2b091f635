"""Drop-in replacements for the reference's hot-path modules (same class names, constructor and
forward signatures, return tuples and state_dict keys as /root/reference/module/*.py)."""
from .STE import SampleGraphSparseGraph  # noqa: F401
from .sbm_attn import Attention, FullAttention, SBMAttention  # noqa: F401
from .disentangled_attn import DisentangledAttn  # noqa: F401
