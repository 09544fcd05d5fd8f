"""Drop-in `GNOT` module backed by the MI355X HIP kernels.

Mirrors the reference interface exactly (aloe101/GNOT-Replication, model.py):
  * same class names and constructor signatures            (model.py:5-7, 33-34, 118-119, 142-143)
  * same submodule structure, hence identical `state_dict` keys, shapes and order, so checkpoints
    saved by main.py:151 load unchanged
  * same forward signature `forward(x, theta, input_functions=None)` -> [B, N, out_dim]
    (model.py:154); input_functions may be the stacked [I, B, M, F] tensor main.py:82 builds or a
    list of [B, M_i, F] tensors
  * same error behaviour: `n_embed should be divisible by head` assertion (model.py:41) and a
    NotImplementedError when input functions are required but not given (model.py:89 calls a
    ModuleList in that case)

Only the whole-model forward/backward runs on the GPU through libgnot_hip.so (one autograd
Function); the submodules exist to own the parameters.  There is no CPU path: on a tensor that is
not on a ROCm device the forward raises.
"""
import weakref

import torch
import torch.nn as nn

from .engine import Engine


class MLP(nn.Module):
    """Parameter container with the reference's layout (model.py:5-18)."""

    def __init__(self, num_layers, input_dim, hidden_dim, output_dim):
        super().__init__()
        layers = [nn.Linear(input_dim, hidden_dim), nn.GELU()]
        for _ in range(num_layers - 1):
            layers += [nn.Linear(hidden_dim, hidden_dim), nn.GELU()]
        layers.append(nn.Linear(hidden_dim, output_dim))
        self.layers = nn.Sequential(*layers)

    def linears(self):
        return [m for m in self.layers if isinstance(m, nn.Linear)]


class LinearAttention(nn.Module):
    """Parameter container of the normalized linear attention (model.py:33-51)."""

    def __init__(self, n_embed, head, n_input_functions=0):
        super().__init__()
        self.head = head
        self.n_embed = n_embed
        self.n_input_functions = n_input_functions
        self.head_dim = n_embed // head
        assert self.head_dim * head == n_embed, "n_embed should be divisible by head"
        self.query = nn.Linear(n_embed, n_embed)
        self.fc_out = nn.Linear(n_embed, n_embed)
        if self.n_input_functions > 0:
            self.key = nn.ModuleList([nn.Linear(n_embed, n_embed) for _ in range(n_input_functions)])
            self.value = nn.ModuleList([nn.Linear(n_embed, n_embed) for _ in range(n_input_functions)])
        else:
            self.key = nn.Linear(n_embed, n_embed)
            self.value = nn.Linear(n_embed, n_embed)

    def linears(self):
        keys = list(self.key) if isinstance(self.key, nn.ModuleList) else [self.key]
        values = list(self.value) if isinstance(self.value, nn.ModuleList) else [self.value]
        return [self.query, self.fc_out] + keys + values


class HeterogeneousNormalizedAttentionBlock(nn.Module):
    """Parameter container of one GNOT block (model.py:118-124)."""

    def __init__(self, n_attn_hidden_dim, n_mlp_num_layers, n_mlp_hidden_dim, n_input_hidden_dim, n_expert,
                 n_head, n_input_functions=0):
        super().__init__()
        self.cross_attention = LinearAttention(n_attn_hidden_dim, n_head, n_input_functions)
        self.self_attention = LinearAttention(n_attn_hidden_dim, n_head)
        self.ffn1 = nn.ModuleList(MLP(n_mlp_num_layers, n_input_hidden_dim, n_mlp_hidden_dim, n_mlp_hidden_dim)
                                  for _ in range(n_expert))
        self.ffn2 = nn.ModuleList(MLP(n_mlp_num_layers, n_input_hidden_dim, n_mlp_hidden_dim, n_mlp_hidden_dim)
                                  for _ in range(n_expert))

    def linears(self):
        out = self.cross_attention.linears() + self.self_attention.linears()
        for m in list(self.ffn1) + list(self.ffn2):
            out += m.linears()
        return out


class _GNOTFunction(torch.autograd.Function):
    """Inputs: (engine, out_dim, n_fns, x, theta, *fns, *weights, *biases).  The backward returns every
    parameter gradient and, when the engine was prepared with input gradients (x, theta or an input
    function requires grad, as the reference's autograd would differentiate them, model.py:154-173),
    the gradients of x, theta and the input functions."""

    @staticmethod
    def forward(ctx, engine, out_dim, nfn, x, theta, *rest):
        fns = list(rest[:nfn])
        P = x.shape[0]
        out = torch.empty(P, out_dim, device=x.device, dtype=torch.float32)
        ctx.engine = engine
        ctx.token = engine.forward(x, theta, fns, out)
        ctx.nfn = nfn
        ctx.in_shapes = (tuple(x.shape), tuple(theta.shape), [tuple(f.shape) for f in fns])
        ctx.nparams = len(rest) - nfn
        return out

    @staticmethod
    def backward(ctx, dout):
        eng = ctx.engine
        if eng.fwd_token != ctx.token:
            raise RuntimeError("gnot_amd: the activations of this forward were reused by a later forward (at most "
                               "GNOT.max_pending_backwards training forwards may await their backward at once; "
                               "raise it with GNOT.set_max_pending_backwards)")
        eng.backward(dout.contiguous().float())
        eng.pending = None
        nfn = ctx.nfn
        need = ctx.needs_input_grad
        in_grads = [None] * (2 + nfn)
        if eng.input_grads and any(need[3:5 + nfn]):
            xs, ts, fs = ctx.in_shapes
            new = lambda shape, want: torch.empty(shape, device=dout.device, dtype=torch.float32) if want else None
            in_grads = [new(xs, need[3]), new(ts, need[4])] + [new(fs[i], need[5 + i]) for i in range(nfn)]
            eng.input_grads_into(in_grads[0], in_grads[1], in_grads[2:])
        head = (None, None, None, *in_grads)
        if not eng.param_grads:
            # the caller consumes the arena itself (gnot_amd.train.FlatAdamW) before the next backward:
            # no copy, and autograd accumulates nothing into .grad
            eng.grad_flat = eng.grad_arena
            return head + (None,) * ctx.nparams
        # ONE copy of the whole gradient arena (the workspace is reused by the next step); every
        # parameter gradient is a view of that fresh buffer
        flat = eng.grad_arena.clone()
        eng.grad_flat = flat        # the step's gradient buffer (sample-DP all-reduces it in place)
        ws, bs = [], []
        for off_w, off_b, shape_w, nb in eng.grad_layout:
            ws.append(flat[off_w:off_w + shape_w[0] * shape_w[1]].view(shape_w))
            bs.append(flat[off_b:off_b + nb])
        # params were passed as (all weights..., all biases...)
        return head + (*ws, *bs)


class GNOT(nn.Module):
    """Drop-in replacement of the reference GNOT (model.py:142-173)."""

    def __init__(self, input_dim, theta_dim, input_func_dim, out_dim, n_attn_layers, n_attn_hidden_dim,
                 n_mlp_num_layers, n_mlp_hidden_dim, n_input_hidden_dim, n_expert, n_head, n_input_functions=0):
        super().__init__()
        self.x = MLP(n_mlp_num_layers, input_dim + theta_dim, n_input_hidden_dim, n_input_hidden_dim)
        self.gating = MLP(n_mlp_num_layers, input_dim, n_mlp_hidden_dim, n_expert)
        self.input_func_mlps = nn.ModuleList(MLP(n_mlp_num_layers, input_func_dim, n_mlp_hidden_dim,
                                                 n_input_hidden_dim) for _ in range(n_input_functions))
        self.blocks = nn.ModuleList(HeterogeneousNormalizedAttentionBlock(
            n_attn_hidden_dim, n_mlp_num_layers, n_mlp_hidden_dim, n_input_hidden_dim, n_expert, n_head,
            n_input_functions) for _ in range(n_attn_layers))
        self.out = MLP(n_mlp_num_layers, n_input_hidden_dim, n_mlp_hidden_dim, out_dim)
        self._cfg = dict(input_dim=input_dim, theta_dim=theta_dim, input_func_dim=input_func_dim,
                         out_dim=out_dim, n_attn_layers=n_attn_layers, n_attn_hidden_dim=n_attn_hidden_dim,
                         n_mlp_num_layers=n_mlp_num_layers, n_mlp_hidden_dim=n_mlp_hidden_dim,
                         n_input_hidden_dim=n_input_hidden_dim, n_expert=n_expert, n_head=n_head,
                         n_input_functions=n_input_functions)
        self._engine = None        # the primary engine: every forward whose predecessor's backward has run
        self._extra = []           # more engines, for forwards issued while earlier ones await their backward
        self.max_pending_backwards = 2
        self._comm = None          # parallel.PointShardComm (set_point_shard); survives engine rebuilds
        self._grad_comm = None     # parallel.PointShardComm (set_grad_allreduce)
        self._moe_recompute = False
        self._bf16 = False

    # canonical Linear order == named_parameters() order of the reference module
    def linears(self):
        out = self.x.linears() + self.gating.linears()
        for m in self.input_func_mlps:
            out += m.linears()
        for blk in self.blocks:
            out += blk.linears()
        return out + self.out.linears()

    def _new_engine(self):
        e = Engine(self._cfg, self.linears())
        e.comm = self._comm
        e.grad_comm = self._grad_comm
        e.moe_recompute = self._moe_recompute
        e.bf16 = self._bf16
        return e

    def engine(self):
        """The primary engine (plan + workspace): the one every forward uses unless an earlier forward's
        backward is still pending on it."""
        if self._engine is None:
            self._engine = self._new_engine()
            self._extra = []
        return self._engine

    def set_max_pending_backwards(self, n):
        """How many training forwards may await their backward at once (default 2).  The reference
        builds a fresh autograd graph per call (model.py:154-173), so `f(a) + f(b)` or gradient
        accumulation over several forwards work there; here every pending forward holds one engine's
        activation set (its own workspace), so this bounds the memory.  A forward beyond the bound
        reuses the oldest pending engine, whose backward then raises."""
        if int(n) < 1:
            raise ValueError("max_pending_backwards must be >= 1")
        self.max_pending_backwards = int(n)

    def _engine_for(self, training):
        """An engine with no pending backward (forwards under no_grad, e.g. an evaluation between a
        training forward and its backward, never disturb a pending one), created on demand; when
        `max_pending_backwards` training forwards are pending, the oldest one's engine."""
        prim = self.engine()
        pool = [prim] + self._extra
        for e in pool:
            if not e.busy():
                return e
        busy = [e for e in pool if e.busy()]
        if training and len(busy) >= self.max_pending_backwards:
            return min(busy, key=lambda e: e.pending_seq)
        e = self._new_engine()
        e.param_grads = prim.param_grads
        e.grad_hook = prim.grad_hook
        self._extra.append(e)
        return e

    def set_precision(self, dtype):
        """'fp32' (default: the reference's fp32 arithmetic, bf16x6-exact on the MFMA) or 'bf16' (BASELINE
        configs[2]'s bf16 training, configs[1]'s "fp32 and bf16": ONE round-to-nearest bf16 operand piece
        per MFMA in the MLP chains, attention projections and weight gradients of every hidden width up to
        256, fp32 accumulation; at d = 256 the soft-MoE expert chains also keep their training saves
        (gelu'(h), expert outputs), dZ and Linear inputs in bf16, which the MoE weight gradients read
        directly; parameters, the other activations and the attention contractions stay fp32).  Above an
        internal width of 256 (d > 256, and the head layouts the d = 256 kernels cannot take, e.g. d = 200 with
        heads of 40: the layer-wise chains) the fp32 path runs in either mode."""
        d = str(dtype).replace("torch.", "")
        if d in ("bf16", "bfloat16"):
            self._bf16 = True
        elif d in ("fp32", "float32", "float"):
            self._bf16 = False
        else:
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {dtype!r}")
        self.engine().bf16 = self._bf16
        self._extra = []           # settings changed: spare engines are rebuilt on demand

    def set_moe_recompute(self, on=True):
        """Memory option (no reference counterpart; torch.utils.checkpoint is the analogue): keep only
        each MoE call's input in training and re-run its expert forward (model.py:128/134) inside the
        backward, so the experts' saved pre-activations exist once instead of once per MoE call.
        Same results; one more MoE forward per call."""
        self._moe_recompute = bool(on)
        self.engine().moe_recompute = self._moe_recompute
        self._extra = []

    def _apply(self, fn, *args, **kwargs):
        # moving / casting the module invalidates the bound parameter pointers
        self._engine = None
        self._extra = []
        return super()._apply(fn, *args, **kwargs)

    def forward(self, x, theta, input_functions=None):
        """Reference calling convention (model.py:154): zero-padded batch x [B, N, input_dim]."""
        B, N, _ = x.shape
        I = self._cfg["n_input_functions"]
        fns, fn_offs = [], []
        if I > 0:
            if input_functions is None:
                # model.py:88-89: the self branch calls the key ModuleList -> NotImplementedError
                raise NotImplementedError("GNOT with n_input_functions > 0 needs input_functions")
            for i in range(I):
                f = input_functions[i]
                M = f.shape[1]
                fns.append(f.reshape(B * M, f.shape[-1]))
                fn_offs.append([b * M for b in range(B + 1)])
        x_off = [b * N for b in range(B + 1)]
        out = self.forward_packed(x.reshape(B * N, x.shape[-1]), x_off, theta, fns, fn_offs)
        return out.view(B, N, -1)

    def set_point_shard(self, comm):
        """Shard every sample's points over the ranks of `comm` (gnot_amd.parallel.PointShardComm), or
        None to switch sharding off.  forward_packed then takes this rank's slices plus n_global."""
        self._comm = comm
        self.engine().comm = comm
        self.engine().geom = None
        self._extra = []

    def set_grad_allreduce(self, comm):
        """Sum the parameter gradients over the ranks of `comm` (gnot_amd.parallel.PointShardComm) INSIDE
        the backward, one collective per weight-gradient group as soon as the group is written, overlapped
        with the rest of the backward (gnot_plan_set_grad_comm); None switches it off (the caller reduces
        the gradients itself, e.g. one all-reduce of engine().grad_flat)."""
        self._grad_comm = comm
        self.engine().grad_comm = comm
        self.engine().geom = None
        self._extra = []

    def forward_packed(self, x, x_off, theta, fns=(), fn_offs=(), n_global=None):
        """Packed-offsets forward (no padding): x [sum N_b, input_dim] with host offsets x_off [B+1];
        fns[i] [sum M_ib, input_func_dim] with fn_offs[i] [B+1].  Equals one B=1 reference call per
        sample, concatenated.  Returns [sum N_b, out_dim].
        Point-sharded (set_point_shard): x holds this rank's slice of every sample (parallel.shard_range)
        and n_global the samples' global point counts; the input functions are passed whole."""
        if not x.is_cuda:
            raise RuntimeError("gnot_amd runs on a ROCm GPU only (libgnot_hip.so); no CPU path")
        x = x.contiguous().float()
        theta = theta.contiguous().float()
        fns = [f.contiguous().float() for f in fns]
        params = [l.weight for l in self.linears()] + [l.bias for l in self.linears()]
        grad = torch.is_grad_enabled()
        inputs_grad = grad and (x.requires_grad or theta.requires_grad or any(f.requires_grad for f in fns))
        training = grad and (inputs_grad or any(p.requires_grad for p in params))
        eng = self._engine_for(training)
        eng.input_grads = inputs_grad
        # every launch (and the plan's side streams) on x's device, whatever device is current
        with torch.cuda.device(x.device):
            eng.prepare([int(v) for v in x_off], [[int(v) for v in o] for o in fn_offs], training, x.device,
                        n_global=None if n_global is None else [int(n) for n in n_global])
            out = _GNOTFunction.apply(eng, self._cfg["out_dim"], len(fns), x, theta, *fns, *params)
        # the engine's activations now belong to this autograd node until its backward runs or the graph is
        # freed (the node is only weakly referenced)
        eng.mark_pending(out.grad_fn if training else None)
        return out
