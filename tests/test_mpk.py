"""burn NamedMpk model files (main.rs:109-116 / training.rs:269-270): the
native loader reads a record written by an independent encoder (python `msgpack`, the layout
restated from burn 0.18 / rmp-serde 1.3 in oracle/mpk_ref.py), the native writer round-trips, and
malformed records are rejected with the field named.  Parity against a file written by the
reference itself is unpinned: the one the reference names is not shipped (.MISSING_LARGE_BLOBS)."""
import numpy as np
import pytest

import azchess as A
import mpk_ref as M


@pytest.mark.parametrize("blocks,filters", [(1, 16), (2, 32)])
def test_loader_reads_independently_encoded_record(tmp_path, blocks, filters):
    w = A.random_weights(blocks, filters, seed=5)
    p = tmp_path / "model.mpk"
    p.write_bytes(M.encode(w, blocks, filters))
    assert np.array_equal(A.load_mpk(p, blocks, filters), w)


def test_f64_elements_and_missing_bias(tmp_path):
    w = A.random_weights(1, 16, seed=6)
    p = tmp_path / "m.mpk"
    p.write_bytes(M.encode(w, 1, 16, f64=True, drop_bias="value_linear_2"))
    got = A.load_mpk(p, 1, 16)
    seg = M.segments(1, 16)
    o = seg["value_linear_2.bias"][0]
    exp = w.copy()
    exp[o] = 0.0                                   # bias: None
    assert np.array_equal(got, exp)


def test_writer_round_trip_and_readable_by_independent_decoder(tmp_path):
    w = A.random_weights(2, 32, seed=7)
    p = tmp_path / "iteration_0_elo_0.mpk"
    A.save_mpk(p, w, 2, 32)                        # what AlphaZero.save_file writes
    assert np.array_equal(A.load_mpk(p, 2, 32), w)
    assert np.array_equal(M.decode(p.read_bytes(), 2, 32), w)


def test_malformed_records_are_rejected(tmp_path):
    w = A.random_weights(1, 16, seed=8)
    p = tmp_path / "bad.mpk"
    p.write_bytes(M.encode(w, 1, 16)[:-10])
    with pytest.raises(A._lib.AzError):
        A.load_mpk(p, 1, 16)
    p.write_bytes(M.encode(w, 1, 16))
    with pytest.raises(A._lib.AzError, match="res_blocks"):
        A.load_mpk(p, 2, 16)                       # wrong architecture
    with pytest.raises(A._lib.AzError, match="shape"):
        A.load_mpk(p, 1, 32)
