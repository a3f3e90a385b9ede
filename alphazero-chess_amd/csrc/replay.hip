// replay.hip -- ReplayBuffer of memory.rs:26-117, host C++ behind the C-ABI.
//
// Entries are keyed by the position's FEN with the pseudo-legal en-passant square
// (memory.rs:42, Fen::from_position(.., EnPassantMode::PseudoLegal)); a position seen again
// folds into a running mean of its improved policy and final value (memory.rs:44-58); a new
// one is appended to a FIFO that evicts the oldest entry at capacity (memory.rs:60-77).
// Sampling draws min(batch, len) distinct entries uniformly (memory.rs:81-101, rand's
// choose_multiple) from a seeded SplitMix64 stream -- the reference's thread_rng is not
// reproducible, so only the distribution is the reference's -- and returns them as network
// inputs (to_tensor planes of the position rebuilt from its FEN, chess.rs:191-245), policies and
// values, ready for az_trainer_step.
// save/load use the reference's on-disk format: bincode 2.0.1 standard config over serde
// (varint lengths and integers, little-endian f32): struct { buffer: HashMap<Fen, MemoryEntry
// { policy: [f32; 4096] (BigArray tuple), value: f32, visit_count: usize }>, order:
// VecDeque<Fen> } with Fen serialised as its string (shakmaty serde).  Restated, not pinned
// against a file the reference wrote (none ships with it).
#include <string.h>

#include <cstdio>
#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

#include "az_internal.h"

struct az_replay {
    struct Entry {
        std::vector<float> policy;   // [4096]
        float value;
        uint64_t visit_count;
    };
    int capacity = 100000;           // REPLAY_BUFFER_SIZE, parameters.rs:10
    std::unordered_map<std::string, Entry> buffer;
    std::deque<std::string> order;
};

using namespace azi;

namespace {

std::string fen_of(const az_pos* p) {
    char buf[128];
    const int n = az_pos_to_fen(p, buf, sizeof(buf));
    return n > 0 ? std::string(buf, n) : std::string();
}

// memory.rs:41-79 with the step's improved policy given densely
int replay_add(az_replay* r, const std::string& key, const float* policy, float value) {
    auto it = r->buffer.find(key);
    if (it != r->buffer.end()) {
        auto& e = it->second;
        const float old_count = (float)e.visit_count;
        const float total = old_count + 1.0f;
        e.value = (e.value * old_count + value) / total;
        for (int i = 0; i < AZ_ACTION_SPACE; i++) e.policy[i] = (e.policy[i] * old_count + policy[i]) / total;
        e.visit_count += 1;
        return 0;
    }
    if ((int)r->order.size() >= r->capacity && !r->order.empty()) {
        r->buffer.erase(r->order.front());
        r->order.pop_front();
    }
    az_replay::Entry e;
    e.policy.assign(policy, policy + AZ_ACTION_SPACE);
    e.value = value;
    e.visit_count = 1;
    r->buffer.emplace(key, std::move(e));
    r->order.push_back(key);
    return 1;
}

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---- bincode 2 standard config
void put_varint(std::string& o, uint64_t v) {
    if (v < 251) { o += (char)v; return; }
    if (v <= 0xFFFF) { o += (char)251; for (int i = 0; i < 2; i++) o += (char)(v >> (8 * i)); return; }
    if (v <= 0xFFFFFFFFull) { o += (char)252; for (int i = 0; i < 4; i++) o += (char)(v >> (8 * i)); return; }
    o += (char)253;
    for (int i = 0; i < 8; i++) o += (char)(v >> (8 * i));
}
void put_f32(std::string& o, float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    for (int i = 0; i < 4; i++) o += (char)(u >> (8 * i));
}
void put_str(std::string& o, const std::string& s) { put_varint(o, s.size()); o += s; }

struct Reader {
    const unsigned char* p; size_t n, i = 0; bool ok = true;
    uint64_t le(int k) {
        if (i + k > n) { ok = false; return 0; }
        uint64_t v = 0;
        for (int j = 0; j < k; j++) v |= (uint64_t)p[i + j] << (8 * j);
        i += k;
        return v;
    }
    uint64_t varint() {
        const uint64_t b = le(1);
        if (b < 251) return b;
        if (b == 251) return le(2);
        if (b == 252) return le(4);
        if (b == 253) return le(8);
        ok = false;                  // 254 = u128: never a length here
        return 0;
    }
    float f32() { const uint32_t u = (uint32_t)le(4); float f; memcpy(&f, &u, 4); return f; }
    std::string str() {
        const uint64_t k = varint();
        if (!ok || i + k > n) { ok = false; return std::string(); }
        std::string s(reinterpret_cast<const char*>(p + i), k);
        i += k;
        return s;
    }
};

}  // namespace

extern "C" {

int az_replay_create(int capacity, az_replay** out) {
    if (!out || capacity < 1) return fail("az_replay_create: bad arguments");
    az_replay* r = new az_replay();
    r->capacity = capacity;
    r->buffer.reserve(std::min(capacity, 1 << 20));
    *out = r;
    return 0;
}

int az_replay_destroy(az_replay* r) { delete r; return 0; }

int az_replay_len(const az_replay* r) { return r ? (int)r->buffer.size() : fail("null"); }

int az_replay_add(az_replay* r, const az_episode_step* st) {
    if (!r || !st || st->nvis < 0 || st->nvis > 224) return fail("az_replay_add: bad arguments");
    // improved policy = visits / sum(visits) over the 4096 entries (tree.rs:110-114, T = 1)
    std::vector<float> pol(AZ_ACTION_SPACE, 0.0f);
    float sum = 0.0f;
    for (int i = 0; i < st->nvis; i++) sum += (float)st->vis_n[i];
    for (int i = 0; i < st->nvis; i++) {
        if (st->vis_idx[i] >= AZ_ACTION_SPACE) return fail("az_replay_add: bad move index");
        pol[st->vis_idx[i]] = (float)st->vis_n[i] / sum;
    }
    return replay_add(r, fen_of(&st->state), pol.data(), st->final_value);
}

int az_replay_add_many(az_replay* r, const az_episode_step* steps, int n) {
    if (!r || n < 0 || (n > 0 && !steps)) return fail("az_replay_add_many: bad arguments");
    int added = 0;
    for (int i = 0; i < n; i++) {   // in order, exactly as n calls of az_replay_add
        const int rc = az_replay_add(r, steps + i);
        if (rc < 0) return rc;
        added += rc;
    }
    return added;
}

int az_replay_add_dense(az_replay* r, const az_pos* state, const float* policy, float value) {
    if (!r || !state || !policy) return fail("null");
    return replay_add(r, fen_of(state), policy, value);
}

int az_replay_sample(az_replay* r, int batch, uint64_t seed, float* planes, float* policy, float* value,
                     az_pos* states) {
    if (!r || batch < 0) return fail("az_replay_sample: bad arguments");
    const int len = (int)r->order.size();
    const int n = std::min(batch, len);
    // partial Fisher-Yates over the FIFO positions: n distinct entries, uniformly
    std::vector<int> idx(len);
    for (int i = 0; i < len; i++) idx[i] = i;
    uint64_t s = seed ^ 0xA0761D6478BD642Full;
    for (int i = 0; i < n; i++) {
        const int j = i + (int)(splitmix(s) % (uint64_t)(len - i));
        std::swap(idx[i], idx[j]);
    }
    for (int k = 0; k < n; k++) {
        const std::string& key = r->order[idx[k]];
        const auto& e = r->buffer.at(key);
        az_pos p;
        if (az_pos_from_fen(key.c_str(), &p) != 0) return -1;   // into_position (memory.rs:95)
        if (states) states[k] = p;
        if (planes) az_pos_encode(&p, planes + (size_t)k * AZ_PLANES * 64);
        if (policy) memcpy(policy + (size_t)k * AZ_ACTION_SPACE, e.policy.data(), AZ_ACTION_SPACE * sizeof(float));
        if (value) value[k] = e.value;
    }
    return n;
}

int az_replay_save(const az_replay* r, const char* path) {
    if (!r || !path) return fail("null");
    std::string o;
    o.reserve(r->order.size() * (AZ_ACTION_SPACE * 4 + 120) + 16);
    put_varint(o, r->buffer.size());
    for (const auto& key : r->order) {        // HashMap order is unspecified; FIFO order here
        const auto& e = r->buffer.at(key);
        put_str(o, key);
        for (int i = 0; i < AZ_ACTION_SPACE; i++) put_f32(o, e.policy[i]);
        put_f32(o, e.value);
        put_varint(o, e.visit_count);
    }
    put_varint(o, r->order.size());
    for (const auto& key : r->order) put_str(o, key);
    FILE* f = fopen(path, "wb");
    if (!f) return fail(std::string("az_replay_save: cannot open ") + path);
    const bool ok = fwrite(o.data(), 1, o.size(), f) == o.size();
    fclose(f);
    return ok ? 0 : fail("az_replay_save: write failed");
}

int az_replay_load(const char* path, int capacity, az_replay** out) {
    if (!path || !out) return fail("null");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(std::string("az_replay_load: cannot open ") + path);
    std::string data;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, k);
    fclose(f);
    Reader rd{reinterpret_cast<const unsigned char*>(data.data()), data.size()};
    az_replay* r = new az_replay();
    r->capacity = capacity > 0 ? capacity : 100000;
    const uint64_t nmap = rd.varint();
    for (uint64_t i = 0; rd.ok && i < nmap; i++) {
        std::string key = rd.str();
        az_replay::Entry e;
        e.policy.resize(AZ_ACTION_SPACE);
        for (int j = 0; j < AZ_ACTION_SPACE; j++) e.policy[j] = rd.f32();
        e.value = rd.f32();
        e.visit_count = rd.varint();
        if (rd.ok) r->buffer[key] = std::move(e);
    }
    const uint64_t nord = rd.ok ? rd.varint() : 0;
    for (uint64_t i = 0; rd.ok && i < nord; i++) r->order.push_back(rd.str());
    if (!rd.ok || rd.i != rd.n || r->order.size() != r->buffer.size()) {
        delete r;
        return fail("az_replay_load: malformed file");
    }
    for (const auto& key : r->order)
        if (!r->buffer.count(key)) { delete r; return fail("az_replay_load: order names a missing entry"); }
    *out = r;
    return 0;
}

}  // extern "C"
