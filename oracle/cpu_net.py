"""Batched f32 forward of AlphaZero (agent.rs:112-144) on the HOST CPU -- the network half of the
CPU baseline, TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and
tests/ use it; the product never does).

burn inference semantics (model.valid(), training.rs:83): BatchNorm from running statistics, folded
into the preceding conv's weights and bias (w' = w * gamma / sqrt(var + 1e-5), b' = (b - mean) *
gamma / sqrt(var + 1e-5) + beta) as an optimised CPU engine would do; the 3x3 / 1x1 convs run through
torch-CPU (oneDNN: blocked direct / im2col GEMM kernels, OpenMP over the host cores) on a
channels-last batch -- one forward over every pending leaf of a simulation step (process_batch,
training.rs:380-422).  Checked against oracle.RefNet within the f32 tolerance (tests)."""
import numpy as np
import torch
import torch.nn.functional as Fn

from train_ref import segments


class CpuNet:
    def __init__(self, blocks, filters, flat, threads=16):
        torch.set_num_threads(threads)
        self.blocks, self.F, self.threads = blocks, filters, threads
        seg, n = segments(blocks, filters)
        flat = np.asarray(flat, np.float32)
        assert flat.size == n

        def get(name):
            o, shape, _ = seg[name]
            return torch.tensor(flat[o:o + int(np.prod(shape))].reshape(shape), dtype=torch.float64)

        def fold(conv, bn):
            w, b = get(conv + ".weight"), get(conv + ".bias")
            g = get(bn)
            s = g[0] / torch.sqrt(g[3] + 1e-5)
            wf = (w * s.reshape(-1, *([1] * (w.dim() - 1)))).float().contiguous(memory_format=torch.channels_last)
            return wf, ((b - g[2]) * s + g[1]).float()

        self.conv = [fold("input_conv", "input_bn")]
        for b in range(blocks):
            self.conv.append(fold("res_blocks.%d.conv1" % b, "res_blocks.%d.bn1" % b))
            self.conv.append(fold("res_blocks.%d.conv2" % b, "res_blocks.%d.bn2" % b))
        self.p1 = fold("policy_conv_1", "policy_bn")
        self.v1 = fold("value_conv", "value_bn")
        self.p2 = (get("policy_conv_2.weight").float(), get("policy_conv_2.bias").float())
        self.l1 = (get("value_linear_1.weight").float(), get("value_linear_1.bias").float())
        self.l2 = (get("value_linear_2.weight").float(), get("value_linear_2.bias").float())

    @torch.inference_mode()
    def forward(self, planes):
        x = torch.from_numpy(np.ascontiguousarray(planes, np.float32).reshape(-1, 19, 8, 8))
        x = x.contiguous(memory_format=torch.channels_last)
        w, b = self.conv[0]
        x = torch.relu(Fn.conv2d(x, w, b, padding=1))
        for k in range(self.blocks):
            r = x
            w, b = self.conv[1 + 2 * k]
            x = torch.relu(Fn.conv2d(x, w, b, padding=1))
            w, b = self.conv[2 + 2 * k]
            x = torch.relu(Fn.conv2d(x, w, b, padding=1) + r)
        p = torch.relu(Fn.conv2d(x, *self.p1))
        p = Fn.conv2d(p, *self.p2).contiguous().reshape(x.shape[0], -1)
        policy = torch.softmax(p, dim=1)
        v = torch.relu(Fn.conv2d(x, *self.v1)).contiguous().reshape(x.shape[0], -1)
        v = torch.relu(v @ self.l1[0] + self.l1[1])
        value = torch.tanh(v @ self.l2[0] + self.l2[1]).squeeze(1)
        return policy.numpy(), value.numpy()
