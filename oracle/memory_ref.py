"""ReplayBuffer oracle -- TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

Pure-Python restatement of memory.rs:26-117: FEN-keyed running means (memory.rs:41-58, float32
arithmetic in the reference's operation order), FIFO eviction at capacity (memory.rs:60-77),
and the bincode 2.0.1 standard-config serde layout of `ReplayBuffer` (memory.rs:107-117):
  varint(len(buffer)), then per entry: str(fen), 4096 x f32 LE (BigArray tuple), f32 value,
  varint(visit_count); then varint(len(order)), str(fen) per entry;
  varint: v < 251 -> 1 byte; <= u16 -> 251 + 2 bytes LE; <= u32 -> 252 + 4; else 253 + 8;
  str: varint(len) + UTF-8 bytes.
Entry order inside the HashMap is unspecified in the reference; written here in FIFO order.
Parity unpinned against a file written by the reference (none ships with it).
"""
import collections
import struct

import numpy as np


class ReplayRef:
    def __init__(self, capacity=100_000):
        self.capacity = capacity
        self.buffer = {}
        self.order = collections.deque()

    def add(self, fen, policy, value):
        policy = np.asarray(policy, np.float32)
        value = np.float32(value)
        if fen in self.buffer:
            pol, val, cnt = self.buffer[fen]
            old = np.float32(cnt)
            tot = np.float32(old + np.float32(1.0))
            val = np.float32(np.float32(val * old + value) / tot)
            pol = ((pol * old + policy) / tot).astype(np.float32)
            self.buffer[fen] = (pol, val, cnt + 1)
            return 0
        if len(self.order) >= self.capacity:
            self.buffer.pop(self.order.popleft())
        self.buffer[fen] = (policy.copy(), value, 1)
        self.order.append(fen)
        return 1

    def __len__(self):
        return len(self.buffer)


def varint(v):
    if v < 251:
        return bytes([v])
    if v <= 0xFFFF:
        return b"\xfb" + struct.pack("<H", v)
    if v <= 0xFFFFFFFF:
        return b"\xfc" + struct.pack("<I", v)
    return b"\xfd" + struct.pack("<Q", v)


def encode(ref):
    out = [varint(len(ref.buffer))]
    for fen in ref.order:
        pol, val, cnt = ref.buffer[fen]
        b = fen.encode()
        out += [varint(len(b)), b, np.asarray(pol, "<f4").tobytes(), struct.pack("<f", val), varint(cnt)]
    out.append(varint(len(ref.order)))
    for fen in ref.order:
        b = fen.encode()
        out += [varint(len(b)), b]
    return b"".join(out)
