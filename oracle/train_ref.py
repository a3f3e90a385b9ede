"""Training-step oracle -- TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

torch-CPU restatement of the reference's train() inner loop for one batch, in float64:
  * forward of agent.rs:112-144 with BatchNorm in TRAINING mode (burn 0.18
    BatchNorm::forward_train, restated: batch mean, biased variance (mean of squared
    deviations), y = ((x - mean) / sqrt(var + 1e-5)) * gamma + beta; running statistics
    updated as rm = rm*0.9 + mean*0.1, rv = rv*0.9 + var*0.1 -- the biased variance, unlike
    torch.nn.BatchNorm2d's unbiased one);
  * compute_gradients (training.rs:277-292): policy_loss = -(t * log(p + 1e-5)).sum(1).mean(),
    value_loss = mean((v - z)^2), loss = policy_loss + 0.5 * value_loss, autograd backward;
  * burn AdamW with GradientClipping::Value(1.0) and weight decay 1e-4 (training.rs:63-66):
    g = clamp(g, -1, 1); m = 0.9m + 0.1g; v = 0.999v + 0.001g^2; p = p*(1 - lr*wd) -
    lr * (m/(1-0.9^t)) / (sqrt(v/(1-0.999^t)) + 1e-5)  (eps outside the sqrt, as burn's
    AdaptiveMomentumW), restated in float32 numpy in the reference's operation order.
burn/cubecl are not vendored and cannot run here: these semantics are restated from burn
0.18's published source -- parity unpinned against burn itself.
Weights use the flat layout of include/az.h (burn module order), restated here independently
of the product's own layout code.
"""
import numpy as np
import torch
import torch.nn.functional as Fn


def param_shapes(blocks, F):
    """(name, shape, is_bn) in the flat order of az_net_num_params (agent.rs:49-110)."""
    out = [("input_conv.weight", (F, 19, 3, 3), False), ("input_conv.bias", (F,), False),
           ("input_bn", (4, F), True)]
    for b in range(blocks):
        for k in (1, 2):
            out += [("res_blocks.%d.conv%d.weight" % (b, k), (F, F, 3, 3), False),
                    ("res_blocks.%d.conv%d.bias" % (b, k), (F,), False),
                    ("res_blocks.%d.bn%d" % (b, k), (4, F), True)]
    out += [("policy_conv_1.weight", (32, F, 1, 1), False), ("policy_conv_1.bias", (32,), False),
            ("policy_bn", (4, 32), True),
            ("policy_conv_2.weight", (64, 32, 1, 1), False), ("policy_conv_2.bias", (64,), False),
            ("value_conv.weight", (8, F, 1, 1), False), ("value_conv.bias", (8,), False),
            ("value_bn", (4, 8), True),
            ("value_linear_1.weight", (512, 64), False), ("value_linear_1.bias", (64,), False),
            ("value_linear_2.weight", (64, 1), False), ("value_linear_2.bias", (1,), False)]
    return out


def segments(blocks, F):
    """name -> (offset, shape, is_bn)"""
    o, seg = 0, {}
    for name, shape, bn in param_shapes(blocks, F):
        seg[name] = (o, shape, bn)
        o += int(np.prod(shape))
    return seg, o


def trainable_mask(blocks, F):
    seg, n = segments(blocks, F)
    m = np.ones(n, bool)
    for name, (o, shape, bn) in seg.items():
        if bn:
            C = shape[1]
            m[o + 2 * C:o + 4 * C] = False
    return m


class TrainRef:
    def __init__(self, blocks, F, flat, dtype=torch.float64):
        self.blocks, self.F, self.dtype = blocks, F, dtype
        self.seg, self.n = segments(blocks, F)
        flat = np.asarray(flat, np.float32)
        assert flat.size == self.n
        self.flat = flat.copy()
        self.P, self.stats = {}, {}
        for name, (o, shape, bn) in self.seg.items():
            a = torch.tensor(flat[o:o + int(np.prod(shape))].reshape(shape), dtype=dtype)
            if bn:
                self.P[name + ".gamma"] = a[0].clone().requires_grad_(True)
                self.P[name + ".beta"] = a[1].clone().requires_grad_(True)
                self.stats[name] = [a[2].clone(), a[3].clone()]
            else:
                self.P[name] = a.clone().requires_grad_(True)

    def _bn(self, x, name):
        mean = x.mean(dim=(0, 2, 3))
        var = ((x - mean[None, :, None, None]) ** 2).mean(dim=(0, 2, 3))
        rm, rv = self.stats[name]
        self.stats[name] = [rm * 0.9 + mean.detach() * 0.1, rv * 0.9 + var.detach() * 0.1]
        std = torch.sqrt(var + 1e-5)
        y = (x - mean[None, :, None, None]) / std[None, :, None, None]
        return y * self.P[name + ".gamma"][None, :, None, None] + self.P[name + ".beta"][None, :, None, None]

    def _conv(self, x, name, pad):
        return Fn.conv2d(x, self.P[name + ".weight"], self.P[name + ".bias"], padding=pad)

    def forward(self, planes, masks=None):
        """masks (optional): ReLU masks in forward order (input block, then per residual block
        the inner and the outer ReLU, heads [B,40,8,8] policy|value, value hidden [B,64]) --
        given, every ReLU multiplies by that mask instead of testing its own sign, so a
        pre-activation within rounding of 0 takes the same branch as in the run that made them."""
        M = None if masks is None else [torch.tensor(np.asarray(m), dtype=self.dtype) for m in masks]

        def relu(z, k, sl=None):
            if M is None:
                return torch.relu(z)
            m = M[k] if sl is None else M[k][:, sl]
            return z * m

        x = torch.tensor(np.asarray(planes, np.float32).reshape(-1, 19, 8, 8), dtype=self.dtype)
        x = relu(self._bn(self._conv(x, "input_conv", 1), "input_bn"), 0)
        for b in range(self.blocks):
            r = x
            x = relu(self._bn(self._conv(x, "res_blocks.%d.conv1" % b, 1), "res_blocks.%d.bn1" % b), 1 + 2 * b)
            x = self._bn(self._conv(x, "res_blocks.%d.conv2" % b, 1), "res_blocks.%d.bn2" % b)
            x = relu(x + r, 2 + 2 * b)
        nh = 2 * self.blocks + 1
        p = relu(self._bn(self._conv(x, "policy_conv_1", 0), "policy_bn"), nh, slice(0, 32))
        p = self._conv(p, "policy_conv_2", 0).reshape(x.shape[0], -1)
        policy = torch.softmax(p, dim=1)
        v = relu(self._bn(self._conv(x, "value_conv", 0), "value_bn"), nh, slice(32, 40)).reshape(x.shape[0], -1)
        v = relu(v @ self.P["value_linear_1.weight"] + self.P["value_linear_1.bias"], nh + 1)
        value = torch.tanh(v @ self.P["value_linear_2.weight"] + self.P["value_linear_2.bias"]).squeeze(1)
        return policy, value

    def grads(self, planes, tpol, tval, masks=None):
        """Returns (flat gradient float64 array, (policy_loss, value_loss)) and leaves the updated
        running statistics in self.stats."""
        for t in self.P.values():
            t.grad = None
        policy, value = self.forward(planes, masks)
        t = torch.tensor(np.asarray(tpol, np.float32), dtype=self.dtype)
        z = torch.tensor(np.asarray(tval, np.float32), dtype=self.dtype)
        pl = -(t * torch.log(policy + 1e-5)).sum(dim=1).mean()
        d = value - z
        vl = (d * d).mean()
        (pl + vl * 0.5).backward()
        g = np.zeros(self.n, np.float64)
        for name, (o, shape, bn) in self.seg.items():
            if bn:
                C = shape[1]
                g[o:o + C] = self.P[name + ".gamma"].grad.numpy()
                g[o + C:o + 2 * C] = self.P[name + ".beta"].grad.numpy()
            else:
                g[o:o + int(np.prod(shape))] = self.P[name].grad.numpy().reshape(-1)
        return g, (float(pl.detach()), float(vl.detach()))

    def running_stats_flat(self, base):
        """`base` (flat) with the running statistics replaced by this oracle's."""
        out = np.array(base, np.float64)
        for name, (o, shape, bn) in self.seg.items():
            if bn:
                C = shape[1]
                out[o + 2 * C:o + 3 * C] = self.stats[name][0].numpy()
                out[o + 3 * C:o + 4 * C] = self.stats[name][1].numpy()
        return out


def powi_f32(x, n):
    """Rust f32::powi as repeated squaring in f32."""
    r, x = np.float32(1.0), np.float32(x)
    while n > 0:
        if n & 1:
            r = np.float32(r * x)
        x = np.float32(x * x)
        n >>= 1
    return r


def adamw_step(p, g, m, v, mask, t, lr, world=1):
    """burn AdamW + value clipping on flat float32 arrays (returns new p, m, v); t = step
    number after increment (1 on the first step)."""
    p, g, m, v = (np.asarray(a, np.float32) for a in (p, g, m, v))
    f = np.float32
    gr = np.clip(g * f(1.0 / world), f(-1.0), f(1.0)).astype(np.float32)
    m1 = (m * f(0.9) + gr * f(np.float32(1.0) - np.float32(0.9))).astype(np.float32)
    m2 = (v * f(0.999) + (gr * gr) * f(np.float32(1.0) - np.float32(0.999))).astype(np.float32)
    bc1 = f(1.0) - powi_f32(0.9, t)
    bc2 = f(1.0) - powi_f32(0.999, t)
    upd = ((m1 / bc1) / (np.sqrt(m2 / bc2) + f(1e-5))).astype(np.float32)
    decay = f(1.0 - lr * 1e-4)
    pn = (p * decay - upd * f(lr)).astype(np.float32)
    return np.where(mask, pn, p), np.where(mask, m1, m), np.where(mask, m2, v)


def cyclical_lr(iteration):
    """get_cyclical_lr (training.rs:424-441) with parameters.rs:20-24."""
    decay = iteration // 1000
    mult = 10.0 ** (-decay)
    base, mx = 1e-3 * mult, 1e-2 * mult
    cur = iteration % 20
    rng = mx - base
    if cur <= 10:
        return base + cur / 10.0 * rng
    return mx - (cur - 10) / 10.0 * rng
