"""C-ABI conformance with the Go shim of INTEGRATION.md (tbls/hipbls.go, never compiled here: the
image has no Go toolchain).

CPU: the shim's status -> error-string switches (verifyStatusErr, verifyAggStatusErr, the switch of
ThresholdAggregateBatch, Aggregate's check) are parsed out of INTEGRATION.md and compared, status by
status, with charon_amd.tbls.STATUS_ERRORS, the table the Python mirror and the caller mirrors use;
the header's enum values are parsed out of include/hipbls.h and compared with charon_amd._lib.

GPU (-m gpu): the shim's exact buffer shapes replayed through ctypes -- sentinel bytes appended to
every blob (sigBlob/idx of ThresholdAggregateBatch, pkBlob of VerifyAggregateBatch, Aggregate's
blob), packMsgs' one-byte blob for all-empty messages, unsafe.Slice over contiguous [N]byte arrays,
sorted share indices, single-item batches and all-empty groups -- with the statuses mapped to
error strings by the parsed Go switches and compared with what herumi returns (the oracle's
fixtures: tests/golden/fixtures_small.json).
"""
import ctypes
import os
import re

import pytest

from charon_amd import _lib, tbls

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return f.read()


def _header_enum():
    """include/hipbls.h enum hbls_status -> {name: value}."""
    body = re.search(r"enum hbls_status \{(.*?)\};", _read("include/hipbls.h"), re.S).group(1)
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"(HBLS_[A-Z_]+)\s*=\s*(\d+)", body)}


def _go_func(src, signature_re):
    """The body of the Go function whose declaration matches signature_re (brace matched)."""
    m = re.search(signature_re, src)
    assert m, signature_re
    i = src.index("{", m.end() - 1)
    depth = 0
    for j in range(i, len(src)):
        depth += {"{": 1, "}": -1}.get(src[j], 0)
        if depth == 0:
            return src[i + 1:j]
    raise AssertionError("unbalanced " + signature_re)


_NEW = re.compile(r'errors\.New\("([^"]*)"\)')


def _parse_switch(body, enum):
    """A Go `switch st... { case C.HBLS_X: ... default: ... }` -> (explicit {status: message or
    None}, default message).  A case without errors.New is the success branch (None)."""
    sw = body[body.index("switch"):]
    explicit, default, cur = {}, None, None
    for line in sw.splitlines()[1:]:
        line = line.strip()
        m = re.match(r"case (.*):$", line)
        if m:
            cur = [enum[c.strip().replace("C.", "")] for c in m.group(1).split(",")]
            for c in cur:
                explicit[c] = None
            continue
        if line == "default:":
            cur = "default"
            continue
        if line == "}":
            break
        n = _NEW.search(line)
        if n and cur is not None:
            if cur == "default":
                default = n.group(1)
            else:
                for c in cur:
                    explicit[c] = n.group(1)
    return explicit, default


def go_status_maps(src=None):
    """kind -> function(status) -> Go error string or None, as the shim in INTEGRATION.md (or the
    text `src`) maps it."""
    src, enum = src or _read("INTEGRATION.md"), _header_enum()
    maps = {}
    for kind, sig in (("verify", r"func verifyStatusErr\(st C\.uint8_t\) error \{"),
                      ("verify_aggregate", r"func verifyAggStatusErr\(st C\.uint8_t\) error \{"),
                      ("threshold_aggregate", r"func \(h HIPBLS\) ThresholdAggregateBatch\([^)]*\) \([^)]*\) \{")):
        explicit, default = _parse_switch(_go_func(src, sig), enum)
        assert default is not None, kind
        maps[kind] = (lambda e, d: (lambda st: e[st] if st in e else d))(explicit, default)
    agg = _go_func(src, r"func \(h HIPBLS\) Aggregate\(signs \[\]Signature\) \(Signature, error\) \{")
    m = re.search(r"if st != C\.HBLS_OK \{\s*return Signature\{\}, " + _NEW.pattern, agg)
    assert m, "Aggregate's status check"
    maps["aggregate"] = (lambda msg: (lambda st: None if st == enum["HBLS_OK"] else msg))(m.group(1))
    return maps


def test_header_enum_matches_python():
    enum = _header_enum()
    assert enum == {"HBLS_OK": _lib.OK, "HBLS_BAD_PUBKEY": _lib.BAD_PUBKEY, "HBLS_BAD_SIGNATURE": _lib.BAD_SIGNATURE,
                    "HBLS_NOT_VERIFIED": _lib.NOT_VERIFIED, "HBLS_COMBINE_FAILED": _lib.COMBINE_FAILED,
                    "HBLS_BAD_SECRET": _lib.BAD_SECRET, "HBLS_BAD_INPUT": _lib.BAD_INPUT,
                    "HBLS_UNCHECKED": _lib.UNCHECKED}


def test_go_status_strings_equal_python_table():
    """Every status code of every call kind maps to the same herumi string in the Go shim and in
    charon_amd.tbls.STATUS_ERRORS (the one table the Python mirrors use)."""
    maps = go_status_maps()
    assert set(maps) == set(tbls.STATUS_ERRORS)
    for kind, go in maps.items():
        for st in range(0, 256):
            assert go(st) == tbls.status_error(kind, st), (kind, st)
    # and the strings are herumi's (tbls/herumi.go:291,296,300 / :325,331,338 / :260,282 / :236)
    assert go_status_maps()["verify"](_lib.NOT_VERIFIED) == "signature not verified"
    assert go_status_maps()["verify_aggregate"](_lib.NOT_VERIFIED) == "signature verification failed"


def test_parser_sees_a_changed_string():
    """The parser is not vacuous: a shim whose switch says something else is caught."""
    src = _read("INTEGRATION.md")
    bad = src.replace('return errors.New("signature not verified")', 'return errors.New("signature NOT verified")', 1)
    assert bad != src
    go = go_status_maps(bad)["verify"]
    assert go(_lib.NOT_VERIFIED) == "signature NOT verified" != tbls.status_error("verify", _lib.NOT_VERIFIED)
    bad = src.replace("case C.HBLS_BAD_SIGNATURE:\n\t\t\terrs[i] = errors.New(", "case C.HBLS_BAD_PUBKEY:\n\t\t\terrs[i] = errors.New(", 1)
    assert bad != src
    go = go_status_maps(bad)["threshold_aggregate"]
    assert go(_lib.BAD_SIGNATURE) != tbls.status_error("threshold_aggregate", _lib.BAD_SIGNATURE)


# ------------------------------------------------------------------------------------- GPU

def _u8(b: bytes):
    return ctypes.create_string_buffer(bytes(b), len(b))


def _arr(ct, xs):
    return (ct * len(xs))(*xs)


def _pack_msgs(msgs):
    """packMsgs: blob, offsets, lengths; a one-byte blob when every message is empty."""
    blob, off, lens = b"", [], []
    for m in msgs:
        off.append(len(blob))
        lens.append(len(m))
        blob += m
    if not blob:
        blob = b"\x00"
    return blob, off, lens


def go_verify_batch(L, pks, msgs, sigs):
    n = len(pks)
    blob, off, lens = _pack_msgs(msgs)
    st = ctypes.create_string_buffer(n)
    # unsafe.Slice(&pks[0][0], 48*n): the [48]byte array elements are contiguous
    rc = L.hbls_verify_batch(_u8(b"".join(pks)), _u8(b"".join(sigs)), _u8(blob), _arr(ctypes.c_uint64, off),
                             _arr(ctypes.c_uint32, lens), n, st)
    assert rc == 0, L.hbls_last_error()
    return list(st.raw[:n])


def go_threshold_aggregate_batch(L, groups):
    g = len(groups)
    sig_blob, idx, grp_off = b"", [], [0] * (g + 1)
    for i, grp in enumerate(groups):
        for k in sorted(grp):  # sort.Ints(keys)
            sig_blob += grp[k]
            idx.append(k)
        grp_off[i + 1] = len(idx)
    sig_blob, idx = sig_blob + b"\x00", idx + [0]  # valid pointers when every group is empty
    out, st = ctypes.create_string_buffer(96 * g), ctypes.create_string_buffer(g)
    rc = L.hbls_threshold_aggregate_batch(_u8(sig_blob), _arr(ctypes.c_int64, idx), _arr(ctypes.c_uint32, grp_off), g,
                                          out, st)
    assert rc == 0, L.hbls_last_error()
    return [out.raw[96 * i:96 * i + 96] for i in range(g)], list(st.raw[:g])


def go_aggregate(L, signs):
    blob = b"".join(signs) + b"\x00"
    out, st = ctypes.create_string_buffer(96), ctypes.create_string_buffer(1)
    rc = L.hbls_aggregate_batch(_u8(blob), _arr(ctypes.c_uint32, [0, len(signs)]), 1, out, st)
    assert rc == 0, L.hbls_last_error()
    return out.raw, st.raw[0]


def go_verify_aggregate_batch(L, keys, sigs, msgs):
    g = len(keys)
    pk_blob, grp_off = b"", [0] * (g + 1)
    for i, k in enumerate(keys):
        pk_blob += b"".join(k)
        grp_off[i + 1] = grp_off[i] + len(k)
    pk_blob += b"\x00"
    blob, off, lens = _pack_msgs(msgs)
    st = ctypes.create_string_buffer(g)
    rc = L.hbls_verify_aggregate_batch(_u8(pk_blob), _arr(ctypes.c_uint32, grp_off), _u8(b"".join(sigs)), _u8(blob),
                                       _arr(ctypes.c_uint64, off), _arr(ctypes.c_uint32, lens), g, st)
    assert rc == 0, L.hbls_last_error()
    return list(st.raw[:g])


@pytest.fixture(scope="module")
def L():
    return _lib.lib()


@pytest.mark.gpu
def test_go_shapes_verify(L, fixtures):
    """VerifyBatch / Verify: the mixed-status fixture batch, every item as its own single-item batch,
    and all-empty messages (packMsgs' one-byte blob); errors as the Go switch maps them."""
    go = go_status_maps()["verify"]
    cs = fixtures["verify"]
    pks = [bytes.fromhex(c["pk"]) for c in cs]
    msgs = [bytes.fromhex(c["msg"]) for c in cs]
    sigs = [bytes.fromhex(c["sig"]) for c in cs]
    want = [tbls.status_error("verify", c["status"]) for c in cs]
    assert [go(s) for s in go_verify_batch(L, pks, msgs, sigs)] == want
    for k in range(len(cs)):  # h.Verify: a one-item batch
        assert go(go_verify_batch(L, [pks[k]], [msgs[k]], [sigs[k]])[0]) == want[k], cs[k]["name"]
    empty = [c for c in cs if c["msg"] == ""]
    assert empty, "the fixtures hold an empty message"
    e = empty[0]
    st = go_verify_batch(L, [bytes.fromhex(e["pk"])] * 3, [b""] * 3, [bytes.fromhex(e["sig"])] * 3)
    assert st == [e["status"]] * 3


@pytest.mark.gpu
def test_go_shapes_threshold_aggregate(L, fixtures):
    """ThresholdAggregateBatch: sorted indices, the sentinel byte and index, all-empty groups,
    single-group calls (h.ThresholdAggregate); outputs byte-equal to the oracle's."""
    go = go_status_maps()["threshold_aggregate"]
    cs = fixtures["threshold_aggregate"]
    groups = [{int(k): bytes.fromhex(v) for k, v in c["partials"].items()} for c in cs]
    outs, sts = go_threshold_aggregate_batch(L, groups)
    for c, o, s in zip(cs, outs, sts):
        assert go(s) == tbls.status_error("threshold_aggregate", c["status"]), c["name"]
        if s == _lib.OK:
            assert o.hex() == c["out"], c["name"]
    for c, grp in zip(cs, groups):
        (o,), (s,) = go_threshold_aggregate_batch(L, [grp])
        assert s == c["status"], c["name"]
        if s == _lib.OK:
            assert o.hex() == c["out"], c["name"]
    empty = {c["name"]: c for c in cs}["empty"]
    _, sts = go_threshold_aggregate_batch(L, [{}, {}, {}])
    assert sts == [empty["status"]] * 3


@pytest.mark.gpu
def test_go_shapes_aggregate_and_verify_aggregate(L, fixtures):
    """Aggregate (trailing sentinel, empty input -> infinity) and VerifyAggregateBatch (sentinel
    after the key blob; a group with no keys; one group per call)."""
    for c in fixtures["aggregate"]:
        out, st = go_aggregate(L, [bytes.fromhex(s) for s in c["sigs"]])
        assert st == c["status"], c["name"]
        assert go_status_maps()["aggregate"](st) == tbls.status_error("aggregate", c["status"])
        if st == _lib.OK:
            assert out.hex() == c["out"], c["name"]
    go = go_status_maps()["verify_aggregate"]
    cs = fixtures["verify_aggregate"]
    keys = [[bytes.fromhex(p) for p in c["pks"]] for c in cs]
    sigs = [bytes.fromhex(c["sig"]) for c in cs]
    msgs = [bytes.fromhex(c["msg"]) for c in cs]
    st = go_verify_aggregate_batch(L, keys, sigs, msgs)
    assert [go(s) for s in st] == [tbls.status_error("verify_aggregate", c["status"]) for c in cs]
    for k, c in enumerate(cs):
        assert go_verify_aggregate_batch(L, [keys[k]], [sigs[k]], [msgs[k]]) == [c["status"]], c["name"]
    no_keys = {c["name"]: c for c in cs}["no_keys"]
    assert go_verify_aggregate_batch(L, [[], []], [sigs[0]] * 2, [msgs[0]] * 2) == [no_keys["status"]] * 2
