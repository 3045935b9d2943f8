"""The C-ABI library loads without a GPU and exports every symbol include/ofr.h declares."""
import os
import re

from opencv_facerecognizer_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "ofr.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(ofr_[a-z0-9_]+)\s*\(", src))


def test_header_matches_bindings():
    assert declared() == set(_lib.SIGNATURES)


def prototypes():
    """name -> number of parameters of every function include/ofr.h declares."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(ofr_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_binding_argument_counts():
    """ctypes passes whatever it is given: a binding with the wrong arity would shift every argument."""
    protos = prototypes()
    assert set(protos) == declared()
    bad = {n: (protos[n], len(_lib.SIGNATURES[n][1])) for n in protos if protos[n] != len(_lib.SIGNATURES[n][1])}
    assert not bad, bad


def test_shard_struct_fields():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    body = re.search(r"typedef struct ofr_knn_shard \{(.*?)\} ofr_knn_shard;", src, flags=re.S).group(1)
    fields = re.findall(r"(\w+);", body)
    assert fields == [f[0] for f in _lib.KnnShard._fields_]


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.ofr_version() == (0 << 16) | (1 << 8)


def test_error_paths_without_device():
    lib = _lib.load()
    # argument validation happens before any device work and reports through ofr_last_error
    rc = lib.ofr_knn_f32(None, 7, None, 1, 32, None, 1, 32, 3, None, 1, 0, None, None, None, 0)
    assert rc == -1 and b"metric" in lib.ofr_last_error()
    rc = lib.ofr_knn_f32(None, 0, None, 1, 32, None, 1, 32, 3, None, 99, 0, None, None, None, 0)
    assert rc == -2 and b"k must be" in lib.ofr_last_error()
    assert lib.ofr_knn_workspace_bytes(4096, 1000000, 1) >= 4096 * (1000000 // 256) * 8 * 8
    # the row sample of the fp6 sieve (round 4): at most ceil(N / 64) rows, no reads past the gallery
    assert lib.ofr_f6_sample_step() == 64
    rc = lib.ofr_f6_sample_rows(None, None, 1000, 32, 32, 0, 17, None, None, 0, None, None, None, None)
    assert rc == -1 and b"past the gallery" in lib.ofr_last_error()
    rc = lib.ofr_f6x2_sample_rows(None, None, 1000, 32, 32, 0, 17, None, 0, None, None, None)
    assert rc == -1 and b"past the gallery" in lib.ofr_last_error()
    assert lib.ofr_f6_sample_rows(None, None, 1000, 32, 32, 16, 16, None, None, 0, None, None, None, None) == 0   # empty
    # column-block scales (round 5): 4-byte aligned tables only
    rc = lib.ofr_f6_block_scales(None, 8, 100, 2)
    assert rc == -1 and b"aligned" in lib.ofr_last_error()
