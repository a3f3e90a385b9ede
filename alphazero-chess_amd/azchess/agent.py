"""agent.rs mirror: AlphaZero network (conv tower + policy/value heads) on libaz.

Weights use the flat f32 layout of include/az.h (burn module order, DESIGN.md "Weights").
`random_weights` is the synthetic random init used by the benchmarks and tests: burn's
default KaimingUniform (gain 1/sqrt(3) => U(-1/sqrt(fan_in), 1/sqrt(fan_in))) for conv and
linear weights and biases (agent.rs:59-84 via burn Conv2dConfig/LinearConfig), BatchNorm
gamma=1, beta=0, running mean 0, var 1, plus a seeded 1e-2 perturbation so that the BN fold
is exercised.
"""
import ctypes as C
import os

import numpy as np

from . import _lib as L
from .parameters import NUM_FILTERS, NUM_RES_BLOCKS, SEED


def num_params(blocks, filters):
    return int(L.lib.az_net_num_params(int(blocks), int(filters)))


def param_shapes(blocks, filters):
    """(name, shape, fan_in or None for BatchNorm) in flat order."""
    F = filters
    out = [("input_conv.weight", (F, 19, 3, 3), 19 * 9), ("input_conv.bias", (F,), 19 * 9),
           ("input_bn", (4, F), None)]
    for b in range(blocks):
        for k in (1, 2):
            out += [("res_blocks.%d.conv%d.weight" % (b, k), (F, F, 3, 3), F * 9),
                    ("res_blocks.%d.conv%d.bias" % (b, k), (F,), F * 9),
                    ("res_blocks.%d.bn%d" % (b, k), (4, F), None)]
    out += [("policy_conv_1.weight", (32, F, 1, 1), F), ("policy_conv_1.bias", (32,), F), ("policy_bn", (4, 32), None),
            ("policy_conv_2.weight", (64, 32, 1, 1), 32), ("policy_conv_2.bias", (64,), 32),
            ("value_conv.weight", (8, F, 1, 1), F), ("value_conv.bias", (8,), F), ("value_bn", (4, 8), None),
            ("value_linear_1.weight", (512, 64), 512), ("value_linear_1.bias", (64,), 512),
            ("value_linear_2.weight", (64, 1), 64), ("value_linear_2.bias", (1,), 64)]
    return out


def random_weights(blocks=NUM_RES_BLOCKS, filters=NUM_FILTERS, seed=SEED, bn_perturb=1e-2):
    rng = np.random.default_rng(seed)
    parts = []
    for _name, shape, fan_in in param_shapes(blocks, filters):
        if fan_in is None:
            c = shape[1]
            g = 1.0 + bn_perturb * rng.uniform(-1, 1, c)
            beta = bn_perturb * rng.uniform(-1, 1, c)
            mean = bn_perturb * rng.uniform(-1, 1, c)
            var = 1.0 + bn_perturb * rng.uniform(-1, 1, c)
            parts.append(np.concatenate([g, beta, mean, var]).astype(np.float32))
        else:
            bound = 1.0 / np.sqrt(fan_in)
            parts.append(rng.uniform(-bound, bound, int(np.prod(shape))).astype(np.float32))
    flat = np.concatenate(parts)
    assert flat.size == num_params(blocks, filters)
    return flat


def load_mpk(path, blocks=NUM_RES_BLOCKS, filters=NUM_FILTERS):
    """NamedMpkFileRecorder::<FullPrecisionSettings>::new().load(path) (main.rs:109-116):
    the record's tensors in the flat layout of include/az.h."""
    out = np.empty(num_params(blocks, filters), np.float32)
    L.check(L.lib.az_net_load_mpk(str(path).encode(), int(blocks), int(filters), L.fptr(out), out.size))
    return out


def save_mpk(path, weights, blocks=NUM_RES_BLOCKS, filters=NUM_FILTERS):
    """model.save_file(path, &NamedMpkFileRecorder::<FullPrecisionSettings>) (training.rs:269-270)."""
    w = np.ascontiguousarray(weights, np.float32)
    L.check(L.lib.az_net_save_mpk(str(path).encode(), int(blocks), int(filters), L.fptr(w), w.size))


def load_model(path, blocks=NUM_RES_BLOCKS, filters=NUM_FILTERS, dtype="f32", device=0):
    """main.rs:109-116: AlphaZero::new().load_record(record)."""
    return AlphaZero(blocks, filters, weights=load_mpk(path, blocks, filters), dtype=dtype, device=device)


class AlphaZero:
    """AlphaZero::new / forward (agent.rs:49-144) with weights resident in HBM."""

    def __init__(self, blocks=NUM_RES_BLOCKS, filters=NUM_FILTERS, weights=None, dtype="f32", device=0,
                 seed=SEED):
        if weights is None:
            weights = random_weights(blocks, filters, seed)
        self.weights = np.ascontiguousarray(weights, np.float32)
        self.blocks, self.filters = blocks, filters
        self.dtype = dtype
        desc = L.AzNetDesc(blocks, filters, L.DTYPE_BF16 if dtype == "bf16" else L.DTYPE_F32)
        h = C.c_void_p()
        L.check(L.lib.az_net_create(C.byref(desc), L.fptr(self.weights), self.weights.size, device, C.byref(h)))
        self._h = h
        # libaz runs the fused tower kernel (f32 or bf16) unless AZ_FUSED_TOWER=0
        self.fused_tower = os.environ.get("AZ_FUSED_TOWER", "1") != "0"

    @property
    def tower_kernel(self):
        """Which kernel evaluates this net (libaz's choice: fused f32 Winograd / f32 direct / bf16)."""
        buf = C.create_string_buffer(128)
        L.check(L.lib.az_net_tower_kernel(self._h, buf, 128))
        return buf.value.decode()

    @property
    def winograd(self):
        return "Winograd" in self.tower_kernel

    def __del__(self):
        try:
            L.lib.az_net_destroy(self._h)
        except Exception:
            pass

    def save_file(self, path):
        save_mpk(path, self.weights, self.blocks, self.filters)

    def forward(self, x):
        """x: [N,19,8,8] float32 -> (policy [N,4096] softmax, value [N] tanh)."""
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 19 * 64)
        n = x.shape[0]
        pol = np.zeros((n, 4096), np.float32)
        val = np.zeros(n, np.float32)
        L.check(L.lib.az_net_forward(self._h, L.fptr(x), n, L.fptr(pol), L.fptr(val)))
        return pol, val
