"""gnot_amd — MI355X-native GNOT core (drop-in for aloe101/GNOT-Replication's model.py).

    from gnot_amd import GNOT
    model = GNOT(input_dim, theta_dim, input_func_dim, out_dim, n_attn_layers, n_attn_hidden_dim,
                 n_mlp_num_layers, n_mlp_hidden_dim, n_input_hidden_dim, n_expert, n_head,
                 n_input_functions).cuda()
"""
from .model import GNOT, MLP, LinearAttention, HeterogeneousNormalizedAttentionBlock  # noqa: F401
from . import _lib  # noqa: F401

__all__ = ["GNOT", "MLP", "LinearAttention", "HeterogeneousNormalizedAttentionBlock"]
