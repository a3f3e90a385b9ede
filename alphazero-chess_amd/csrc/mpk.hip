// mpk.hip -- burn NamedMpkFileRecorder<FullPrecisionSettings> model files:
// load_model (main.rs:109-116) and model.save_file (training.rs:269-270) for the AlphaZero
// module of agent.rs, converted from / to the flat parameter layout of include/az.h.
//
// The file is rmp-serde `write_named` (MessagePack, structs as maps keyed by field name) of
// BurnRecord { metadata: { float, int, format, version, settings }, item }, where item is the
// module's record: AlphaZero { input_conv, input_bn, res_blocks: [ { conv1, bn1, conv2, bn2 } ],
// policy_conv_1, policy_bn, policy_conv_2, value_conv, value_bn, value_linear_1,
// value_linear_2 }; Conv2d / Linear { weight, bias (Option) , ... }, BatchNorm { gamma, beta,
// running_mean, running_var, ... }; every tensor is ParamSerde { id, param: TensorData {
// bytes (f32 little-endian at full precision), shape, dtype } }.  The loader walks the tree by
// field name, ignores fields it does not need (stride, padding, momentum, ...), accepts f32 or
// f64 element bytes, and checks every shape against the architecture.  burn 0.18 / rmp-serde
// 1.3 restated from their published sources; no reference-written .mpk ships
// (.MISSING_LARGE_BLOBS), so parity against a real file is unpinned.
#include <math.h>
#include <string.h>

#include <cstdio>
#include <string>
#include <vector>

#include "az_internal.h"

using namespace azi;

namespace {

// ------------------------------------------------------------------ MessagePack tree
struct MV {
    enum Kind { NIL, BOOL, INT, FLOAT, STR, BIN, ARR, MAP } kind = NIL;
    int64_t i = 0;
    double f = 0.0;
    std::string s;                                  // STR and BIN payloads
    std::vector<MV> arr;
    std::vector<std::pair<std::string, MV>> map;    // string keys only (named records)
    const MV* get(const char* k) const {
        if (kind != MAP) return nullptr;
        for (const auto& kv : map)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct Parser {
    const unsigned char* p; size_t n, i = 0; bool ok = true; int depth = 0;
    uint64_t be(int k) {
        if (i + k > n) { ok = false; return 0; }
        uint64_t v = 0;
        for (int j = 0; j < k; j++) v = (v << 8) | p[i + j];
        i += k;
        return v;
    }
    void bytes(size_t k, std::string& out) {
        if (i + k > n) { ok = false; return; }
        out.assign(reinterpret_cast<const char*>(p + i), k);
        i += k;
    }
    MV value() {
        MV v;
        if (!ok || ++depth > 64) { ok = false; return v; }
        const unsigned b = (unsigned)be(1);
        if (b <= 0x7f) { v.kind = MV::INT; v.i = b; }
        else if (b >= 0xe0) { v.kind = MV::INT; v.i = (int8_t)b; }
        else if ((b & 0xf0) == 0x80) map_body(v, b & 0x0f);
        else if ((b & 0xf0) == 0x90) arr_body(v, b & 0x0f);
        else if ((b & 0xe0) == 0xa0) { v.kind = MV::STR; bytes(b & 0x1f, v.s); }
        else switch (b) {
            case 0xc0: break;
            case 0xc2: v.kind = MV::BOOL; v.i = 0; break;
            case 0xc3: v.kind = MV::BOOL; v.i = 1; break;
            case 0xc4: v.kind = MV::BIN; bytes(be(1), v.s); break;
            case 0xc5: v.kind = MV::BIN; bytes(be(2), v.s); break;
            case 0xc6: v.kind = MV::BIN; bytes(be(4), v.s); break;
            case 0xca: { v.kind = MV::FLOAT; const uint32_t u = (uint32_t)be(4); float f; memcpy(&f, &u, 4); v.f = f; break; }
            case 0xcb: { v.kind = MV::FLOAT; const uint64_t u = be(8); double d; memcpy(&d, &u, 8); v.f = d; break; }
            case 0xcc: v.kind = MV::INT; v.i = (int64_t)be(1); break;
            case 0xcd: v.kind = MV::INT; v.i = (int64_t)be(2); break;
            case 0xce: v.kind = MV::INT; v.i = (int64_t)be(4); break;
            case 0xcf: v.kind = MV::INT; v.i = (int64_t)be(8); break;
            case 0xd0: v.kind = MV::INT; v.i = (int8_t)be(1); break;
            case 0xd1: v.kind = MV::INT; v.i = (int16_t)be(2); break;
            case 0xd2: v.kind = MV::INT; v.i = (int32_t)be(4); break;
            case 0xd3: v.kind = MV::INT; v.i = (int64_t)be(8); break;
            case 0xd9: v.kind = MV::STR; bytes(be(1), v.s); break;
            case 0xda: v.kind = MV::STR; bytes(be(2), v.s); break;
            case 0xdb: v.kind = MV::STR; bytes(be(4), v.s); break;
            case 0xdc: arr_body(v, be(2)); break;
            case 0xdd: arr_body(v, be(4)); break;
            case 0xde: map_body(v, be(2)); break;
            case 0xdf: map_body(v, be(4)); break;
            case 0xd4: i += 2; break;                   // fixext 1..16, ext 8/16/32: skipped
            case 0xd5: i += 3; break;
            case 0xd6: i += 5; break;
            case 0xd7: i += 9; break;
            case 0xd8: i += 17; break;
            case 0xc7: { const size_t k = be(1); i += 1 + k; break; }
            case 0xc8: { const size_t k = be(2); i += 1 + k; break; }
            case 0xc9: { const size_t k = be(4); i += 1 + k; break; }
            default: ok = false;
        }
        if (i > n) ok = false;
        depth--;
        return v;
    }
    void arr_body(MV& v, uint64_t k) {
        v.kind = MV::ARR;
        if (k > n - i) { ok = false; return; }
        for (uint64_t j = 0; ok && j < k; j++) v.arr.push_back(value());
    }
    void map_body(MV& v, uint64_t k) {
        v.kind = MV::MAP;
        if (k > n - i) { ok = false; return; }
        for (uint64_t j = 0; ok && j < k; j++) {
            MV key = value();
            MV val = value();
            if (key.kind == MV::STR) v.map.emplace_back(key.s, std::move(val));
            else if (key.kind == MV::INT) v.map.emplace_back(std::to_string(key.i), std::move(val));
            else ok = false;
        }
    }
};

// ------------------------------------------------------------------ writer
struct Writer {
    std::string o;
    void be(uint64_t v, int k) { for (int j = k - 1; j >= 0; j--) o += (char)(v >> (8 * j)); }
    void map(size_t k) { if (k < 16) o += (char)(0x80 | k); else { o += (char)0xde; be(k, 2); } }
    void arr(size_t k) { if (k < 16) o += (char)(0x90 | k); else if (k <= 0xFFFF) { o += (char)0xdc; be(k, 2); } else { o += (char)0xdd; be(k, 4); } }
    void str(const std::string& s) {
        if (s.size() < 32) o += (char)(0xa0 | s.size());
        else if (s.size() <= 0xFF) { o += (char)0xd9; be(s.size(), 1); }
        else { o += (char)0xda; be(s.size(), 2); }
        o += s;
    }
    void bin(const void* d, size_t k) { o += (char)0xc6; be(k, 4); o.append(reinterpret_cast<const char*>(d), k); }
    void uint(uint64_t v) {
        if (v < 128) o += (char)v;
        else if (v <= 0xFF) { o += (char)0xcc; be(v, 1); }
        else if (v <= 0xFFFF) { o += (char)0xcd; be(v, 2); }
        else if (v <= 0xFFFFFFFFull) { o += (char)0xce; be(v, 4); }
        else { o += (char)0xcf; be(v, 8); }
    }
    void f64(double d) { uint64_t u; memcpy(&u, &d, 8); o += (char)0xcb; be(u, 8); }
    void nil() { o += (char)0xc0; }
};

// ------------------------------------------------------------------ AlphaZero record <-> flat
struct Cursor {       // walks the flat layout in burn module order
    const float* in = nullptr; float* out = nullptr; size_t off = 0, n = 0;
};

std::string g_fail;

// TensorData at `node` (ParamSerde {id, param: {bytes, shape, dtype}}, or the TensorData itself)
bool read_tensor(const MV* node, const std::vector<int64_t>& shape, float* dst, const std::string& what) {
    if (!node) { g_fail = "missing tensor " + what; return false; }
    if (const MV* p = node->get("param")) return read_tensor(p, shape, dst, what);
    if (const MV* d = node->get("data")) return read_tensor(d, shape, dst, what);
    const MV* b = node->get("bytes");
    const MV* s = node->get("shape");
    if (!b || !s || s->kind != MV::ARR || (b->kind != MV::BIN && b->kind != MV::ARR)) {
        g_fail = "malformed tensor " + what;
        return false;
    }
    size_t cnt = 1;
    if (s->arr.size() != shape.size()) { g_fail = "rank mismatch for " + what; return false; }
    for (size_t j = 0; j < shape.size(); j++) {
        if (s->arr[j].kind != MV::INT || s->arr[j].i != shape[j]) { g_fail = "shape mismatch for " + what; return false; }
        cnt *= (size_t)shape[j];
    }
    std::string raw;
    if (b->kind == MV::BIN) raw = b->s;
    else for (const auto& e : b->arr) raw += (char)(e.i & 0xFF);     // bytes as an integer sequence
    if (raw.size() == cnt * 4) {
        memcpy(dst, raw.data(), cnt * 4);
    } else if (raw.size() == cnt * 8) {
        for (size_t j = 0; j < cnt; j++) { double d; memcpy(&d, raw.data() + 8 * j, 8); dst[j] = (float)d; }
    } else {
        g_fail = "element size of " + what + " is neither f32 nor f64";
        return false;
    }
    return true;
}

const MV* field(const MV* node, const char* k) { return node ? node->get(k) : nullptr; }

// layer loaders in the flat order of az_net_num_params
bool conv_in(const MV* m, int co, int ci, int k, Cursor& c, const std::string& name) {
    if (!read_tensor(field(m, "weight"), {co, ci, k, k}, c.out + c.off, name + ".weight")) return false;
    c.off += (size_t)co * ci * k * k;
    const MV* b = field(m, "bias");
    if (b && b->kind != MV::NIL) { if (!read_tensor(b, {co}, c.out + c.off, name + ".bias")) return false; }
    else memset(c.out + c.off, 0, co * sizeof(float));                 // bias: None
    c.off += co;
    return true;
}
bool bn_in(const MV* m, int C, Cursor& c, const std::string& name) {
    const char* f[4] = {"gamma", "beta", "running_mean", "running_var"};
    for (int j = 0; j < 4; j++) {
        if (!read_tensor(field(m, f[j]), {C}, c.out + c.off, name + "." + f[j])) return false;
        c.off += C;
    }
    return true;
}
bool linear_in(const MV* m, int din, int dout, Cursor& c, const std::string& name) {
    if (!read_tensor(field(m, "weight"), {din, dout}, c.out + c.off, name + ".weight")) return false;
    c.off += (size_t)din * dout;
    const MV* b = field(m, "bias");
    if (b && b->kind != MV::NIL) { if (!read_tensor(b, {dout}, c.out + c.off, name + ".bias")) return false; }
    else memset(c.out + c.off, 0, dout * sizeof(float));
    c.off += dout;
    return true;
}

int64_t g_id = 0;
void tensor_out(Writer& w, const std::vector<int64_t>& shape, const float* src) {
    size_t cnt = 1;
    for (auto d : shape) cnt *= (size_t)d;
    w.map(2);
    w.str("id");
    char id[32];
    snprintf(id, sizeof(id), "%016llx", (unsigned long long)(0x9E3779B97F4A7C15ull * (uint64_t)++g_id));
    w.str(id);
    w.str("param");
    w.map(3);
    w.str("bytes"); w.bin(src, cnt * 4);
    w.str("shape"); w.arr(shape.size()); for (auto d : shape) w.uint((uint64_t)d);
    w.str("dtype"); w.str("F32");
}
void conv_out(Writer& w, int co, int ci, int k, Cursor& c) {
    w.map(7);
    w.str("weight"); tensor_out(w, {co, ci, k, k}, c.in + c.off); c.off += (size_t)co * ci * k * k;
    w.str("bias"); tensor_out(w, {co}, c.in + c.off); c.off += co;
    w.str("stride"); w.arr(2); w.uint(1); w.uint(1);
    w.str("kernel_size"); w.arr(2); w.uint(k); w.uint(k);
    w.str("dilation"); w.arr(2); w.uint(1); w.uint(1);
    w.str("groups"); w.uint(1);
    w.str("padding"); w.nil();
}
void bn_out(Writer& w, int C, Cursor& c) {
    w.map(6);
    const char* f[4] = {"gamma", "beta", "running_mean", "running_var"};
    for (int j = 0; j < 4; j++) { w.str(f[j]); tensor_out(w, {C}, c.in + c.off); c.off += C; }
    w.str("momentum"); w.f64(0.1);
    w.str("epsilon"); w.f64(1e-5);
}
void linear_out(Writer& w, int din, int dout, Cursor& c) {
    w.map(2);
    w.str("weight"); tensor_out(w, {din, dout}, c.in + c.off); c.off += (size_t)din * dout;
    w.str("bias"); tensor_out(w, {dout}, c.in + c.off); c.off += dout;
}

}  // namespace

extern "C" {

int az_net_load_mpk(const char* path, int blocks, int filters, float* out, size_t n) {
    if (!path || !out || n != az_net_num_params(blocks, filters)) return fail("az_net_load_mpk: bad arguments");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(std::string("az_net_load_mpk: cannot open ") + path);
    std::string data;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, k);
    fclose(f);
    Parser ps{reinterpret_cast<const unsigned char*>(data.data()), data.size()};
    MV root = ps.value();
    if (!ps.ok || ps.i != ps.n) return fail("az_net_load_mpk: not a MessagePack document");
    const MV* item = root.get("item") ? root.get("item") : &root;    // BurnRecord { metadata, item }
    const int F = filters;
    Cursor c;
    c.out = out;
    g_fail.clear();
    bool ok = conv_in(field(item, "input_conv"), F, 19, 3, c, "input_conv") && bn_in(field(item, "input_bn"), F, c, "input_bn");
    const MV* rb = field(item, "res_blocks");
    if (ok && (!rb || rb->kind != MV::ARR || (int)rb->arr.size() != blocks)) {
        g_fail = "res_blocks: expected " + std::to_string(blocks) + " blocks";
        ok = false;
    }
    for (int b = 0; ok && b < blocks; b++) {
        const MV* B = &rb->arr[b];
        const std::string nm = "res_blocks." + std::to_string(b);
        ok = conv_in(field(B, "conv1"), F, F, 3, c, nm + ".conv1") && bn_in(field(B, "bn1"), F, c, nm + ".bn1") &&
             conv_in(field(B, "conv2"), F, F, 3, c, nm + ".conv2") && bn_in(field(B, "bn2"), F, c, nm + ".bn2");
    }
    ok = ok && conv_in(field(item, "policy_conv_1"), 32, F, 1, c, "policy_conv_1") &&
         bn_in(field(item, "policy_bn"), 32, c, "policy_bn") &&
         conv_in(field(item, "policy_conv_2"), 64, 32, 1, c, "policy_conv_2") &&
         conv_in(field(item, "value_conv"), 8, F, 1, c, "value_conv") && bn_in(field(item, "value_bn"), 8, c, "value_bn") &&
         linear_in(field(item, "value_linear_1"), 512, 64, c, "value_linear_1") &&
         linear_in(field(item, "value_linear_2"), 64, 1, c, "value_linear_2");
    if (!ok) return fail("az_net_load_mpk: " + g_fail);
    if (c.off != n) return fail("az_net_load_mpk: layout size mismatch");
    return 0;
}

int az_net_save_mpk(const char* path, int blocks, int filters, const float* w, size_t n) {
    if (!path || !w || n != az_net_num_params(blocks, filters)) return fail("az_net_save_mpk: bad arguments");
    const int F = filters;
    Writer wr;
    Cursor c;
    c.in = w;
    g_id = 0;
    wr.map(2);
    wr.str("metadata");
    wr.map(5);
    wr.str("float"); wr.str("f32");
    wr.str("int"); wr.str("i64");
    wr.str("format"); wr.str("burn::record::file::NamedMpkFileRecorder<burn::record::settings::FullPrecisionSettings>");
    wr.str("version"); wr.str("0.18.0");
    wr.str("settings"); wr.str("FullPrecisionSettings");
    wr.str("item");
    wr.map(10);
    wr.str("input_conv"); conv_out(wr, F, 19, 3, c);
    wr.str("input_bn"); bn_out(wr, F, c);
    wr.str("res_blocks"); wr.arr(blocks);
    for (int b = 0; b < blocks; b++) {
        wr.map(4);
        wr.str("conv1"); conv_out(wr, F, F, 3, c);
        wr.str("bn1"); bn_out(wr, F, c);
        wr.str("conv2"); conv_out(wr, F, F, 3, c);
        wr.str("bn2"); bn_out(wr, F, c);
    }
    wr.str("policy_conv_1"); conv_out(wr, 32, F, 1, c);
    wr.str("policy_bn"); bn_out(wr, 32, c);
    wr.str("policy_conv_2"); conv_out(wr, 64, 32, 1, c);
    wr.str("value_conv"); conv_out(wr, 8, F, 1, c);
    wr.str("value_bn"); bn_out(wr, 8, c);
    wr.str("value_linear_1"); linear_out(wr, 512, 64, c);
    wr.str("value_linear_2"); linear_out(wr, 64, 1, c);
    if (c.off != n) return fail("az_net_save_mpk: layout size mismatch");
    FILE* f = fopen(path, "wb");
    if (!f) return fail(std::string("az_net_save_mpk: cannot open ") + path);
    const bool ok = fwrite(wr.o.data(), 1, wr.o.size(), f) == wr.o.size();
    fclose(f);
    return ok ? 0 : fail("az_net_save_mpk: write failed");
}

}  // extern "C"
