"""NamedMpk record encoder/decoder -- TEST INFRASTRUCTURE ONLY (tests/ may import it).

Independent restatement (python `msgpack`) of the file burn 0.18's
NamedMpkFileRecorder<FullPrecisionSettings> writes for agent.rs' AlphaZero module:
rmp_serde::encode::write_named of BurnRecord { metadata, item }, structs as maps keyed by field
name, tensors as ParamSerde { id, param: TensorData { bytes, shape, dtype } } with f32
little-endian bytes.  Not pinned against a reference-written file (none ships)."""
import msgpack
import numpy as np


def param_shapes(blocks, F):
    out = [("input_conv.weight", (F, 19, 3, 3)), ("input_conv.bias", (F,)), ("input_bn", (4, F))]
    for b in range(blocks):
        for k in (1, 2):
            out += [("res_blocks.%d.conv%d.weight" % (b, k), (F, F, 3, 3)), ("res_blocks.%d.conv%d.bias" % (b, k), (F,)),
                    ("res_blocks.%d.bn%d" % (b, k), (4, F))]
    out += [("policy_conv_1.weight", (32, F, 1, 1)), ("policy_conv_1.bias", (32,)), ("policy_bn", (4, 32)),
            ("policy_conv_2.weight", (64, 32, 1, 1)), ("policy_conv_2.bias", (64,)),
            ("value_conv.weight", (8, F, 1, 1)), ("value_conv.bias", (8,)), ("value_bn", (4, 8)),
            ("value_linear_1.weight", (512, 64)), ("value_linear_1.bias", (64,)),
            ("value_linear_2.weight", (64, 1)), ("value_linear_2.bias", (1,))]
    return out


def segments(blocks, F):
    o, seg = 0, {}
    for name, shape in param_shapes(blocks, F):
        seg[name] = (o, shape)
        o += int(np.prod(shape))
    return seg


def _tensor(a, shape, f64, ident):
    arr = np.asarray(a, np.float64 if f64 else np.float32).reshape(shape)
    return {"id": "%016x" % ident, "param": {"bytes": arr.astype("<f8" if f64 else "<f4").tobytes(),
                                            "shape": list(shape), "dtype": "F64" if f64 else "F32"}}


def encode(w, blocks, F, f64=False, drop_bias=None):
    seg = segments(blocks, F)
    ids = iter(range(1, 10 ** 6))

    def t(name, shape=None):
        o, sh = seg[name]
        sh = shape or sh
        return _tensor(w[o:o + int(np.prod(sh))], sh, f64, next(ids))

    def conv(n):
        d = {"weight": t(n + ".weight"), "bias": None if drop_bias == n else t(n + ".bias"), "stride": [1, 1],
             "kernel_size": [seg[n + ".weight"][1][2]] * 2, "dilation": [1, 1], "groups": 1, "padding": None}
        return d

    def bn(n):
        o, (_, C) = seg[n]
        names = ["gamma", "beta", "running_mean", "running_var"]
        d = {k: _tensor(w[o + j * C:o + (j + 1) * C], (C,), f64, next(ids)) for j, k in enumerate(names)}
        d.update({"momentum": 0.1, "epsilon": 1e-5})
        return d

    def linear(n):
        return {"weight": t(n + ".weight"), "bias": None if drop_bias == n else t(n + ".bias")}

    item = {"input_conv": conv("input_conv"), "input_bn": bn("input_bn"),
            "res_blocks": [{"conv1": conv("res_blocks.%d.conv1" % b), "bn1": bn("res_blocks.%d.bn1" % b),
                            "conv2": conv("res_blocks.%d.conv2" % b), "bn2": bn("res_blocks.%d.bn2" % b)}
                           for b in range(blocks)],
            "policy_conv_1": conv("policy_conv_1"), "policy_bn": bn("policy_bn"), "policy_conv_2": conv("policy_conv_2"),
            "value_conv": conv("value_conv"), "value_bn": bn("value_bn"),
            "value_linear_1": linear("value_linear_1"), "value_linear_2": linear("value_linear_2")}
    rec = {"metadata": {"float": "f64" if f64 else "f32", "int": "i64",
                        "format": "burn::record::file::NamedMpkFileRecorder", "version": "0.18.0",
                        "settings": "FullPrecisionSettings"}, "item": item}
    return msgpack.packb(rec, use_bin_type=True)


def decode(raw, blocks, F):
    rec = msgpack.unpackb(raw, raw=False)
    item = rec["item"]
    seg = segments(blocks, F)
    out = np.zeros(sum(int(np.prod(s)) for _, s in param_shapes(blocks, F)), np.float32)

    def node(name):
        parts = name.split(".")
        cur = item
        for p in parts:
            cur = cur[int(p)] if isinstance(cur, list) else cur[p]
        return cur

    for name, (o, shape) in seg.items():
        if name.endswith("bn") or name.split(".")[-1].startswith("bn"):
            C = shape[1]
            d = node(name)
            for j, k in enumerate(["gamma", "beta", "running_mean", "running_var"]):
                out[o + j * C:o + (j + 1) * C] = np.frombuffer(d[k]["param"]["bytes"], "<f4")
        else:
            d = node(name)
            out[o:o + int(np.prod(shape))] = np.frombuffer(d["param"]["bytes"], "<f4")
    return out
