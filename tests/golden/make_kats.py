"""Extract the reference's BLS known-answer vectors into tests/golden/kat_reference.json.

Run here (where /root/reference exists); the JSON is committed so tests never read the
reference at run time.  Only DATA is extracted (keys, messages, signatures the reference's
own tests hold); signing roots are re-derived with our own SSZ code (oracle/ssz.py) and
cross-checked against the values the reference files state where they state one.

Sources:
  * eth2util/signing/signing_test.go:24-74  (teku-produced registration; sk, pk, sig, domain)
  * eth2util/deposit/deposit_test.go:215-259 + testdata/TestMarshalDepositData.golden
  * cluster/examples/cluster-lock-00{0..3}.json  (cluster/cluster_test.go:242-260 TestExamples)
  * core/testdata/TestSSZSerialisation_{SignedAggregateAndProof, SignedSyncContributionAndProof,
    SyncContributionAndProof, SignedSyncMessage, SignedVoluntaryExit}.ssz.golden and the JSON goldens
    of BeaconCommitteeSelection / SyncCommitteeSelection / SignedRandao, plus the teku registration
    message: the other duty types' objects, each checked
    against its JSON twin; their object roots re-derived with oracle/ssz.py (duty_roots_kats)
  * core/testdata/TestSSZSerialisation_AttestationData.ssz.golden + the .json.golden of the same
    value (core/ssz_test.go): the SSZ bytes of one phase0.AttestationData, cross-checked field by
    field against the JSON; its hash-tree-root is re-derived with oracle/ssz.py (no reference
    file states one)
"""

from __future__ import annotations

import base64
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import ssz  # noqa: E402

REF = "/root/reference"


def _b(v: str) -> bytes:
    if v.startswith("0x"):
        return bytes.fromhex(v[2:])
    return base64.b64decode(v)


def registration_kat():
    src = open(os.path.join(REF, "eth2util/signing/signing_test.go")).read()
    sk = re.search(r'hex.DecodeString\("([0-9a-f]{64})"\)', src).group(1)
    fee = re.search(r'"fee_recipient": "0x([0-9a-fA-F]{40})"', src).group(1)
    gas = int(re.search(r'"gas_limit": "(\d+)"', src).group(1))
    ts = int(re.search(r'"timestamp": "(\d+)"', src).group(1))
    pk = re.search(r'"pubkey": "0x([0-9a-f]{96})"', src).group(1)
    sig = re.search(r'"signature": "0x([0-9a-f]{192})"', src).group(1)
    # expected domain literal (TestConstantApplicationBuilder)
    dom_lit = re.search(r"expect := eth2p0.Domain\{(.*?)\}", src, re.S).group(1)
    dom = bytes(int(x, 16) for x in re.findall(r"0x([0-9a-f]+)", dom_lit))
    fork = bytes.fromhex("01017000")  # holesky genesis, eth2util/network.go:78
    domain = ssz.compute_domain(ssz.DOMAIN_APPLICATION_BUILDER, fork)
    assert domain == dom, "domain derivation disagrees with signing_test.go literal"
    root = ssz.validator_registration_root(bytes.fromhex(fee), gas, ts, bytes.fromhex(pk))
    msg = ssz.signing_root(root, domain)
    # NOTE: "msg_pubkey" is the validator pubkey INSIDE the registration message; the test
    # signs with a secret *share* whose public key the reference derives via SecretToPublicKey.
    return {"source": "eth2util/signing/signing_test.go:24-74", "sk": sk, "msg_pubkey": pk, "msg": msg.hex(),
            "sig": sig, "domain": domain.hex()}


def deposit_kats():
    src = open(os.path.join(REF, "eth2util/deposit/deposit_test.go")).read()
    block = re.search(r"privKeys := \[\]string\{(.*?)\}", src, re.S).group(1)
    sks = re.findall(r'"([0-9a-f]{64})"', block)
    block = re.search(r"withdrawalAddrs := \[\]string\{(.*?)\}", src, re.S).group(1)
    addrs = [a.lower() for a in re.findall(r'"0x([0-9a-fA-F]{40})"', block)]
    golden = json.load(open(os.path.join(REF, "eth2util/deposit/testdata/TestMarshalDepositData.golden")))
    fork = bytes.fromhex("00001020")  # goerli, eth2util/network.go:49
    domain = ssz.compute_domain(ssz.DOMAIN_DEPOSIT, fork)
    out = []
    for g in golden:
        creds = bytes.fromhex(g["withdrawal_credentials"])
        addr = creds[12:].hex()
        sk = sks[addrs.index(addr)]
        mroot = ssz.deposit_message_root(bytes.fromhex(g["pubkey"]), creds, g["amount"])
        assert mroot.hex() == g["deposit_message_root"], "deposit message root mismatch"
        msg = ssz.signing_root(mroot, domain)
        out.append({"source": "eth2util/deposit/testdata/TestMarshalDepositData.golden", "sk": sk,
                    "pk": g["pubkey"], "msg": msg.hex(), "sig": g["signature"]})
    return out


def lock_kats():
    out = []
    for i in range(4):
        path = os.path.join(REF, f"cluster/examples/cluster-lock-00{i}.json")
        d = json.load(open(path))
        dfn = d["cluster_definition"]
        vals = []
        for v in d["distributed_validators"]:
            ent = {"dpk": _b(v["distributed_public_key"]).hex(),
                   "shares": [_b(s).hex() for s in v["public_shares"]]}
            br = v.get("builder_registration")
            if br and br.get("signature"):
                m = br["message"]
                fork = _b(dfn["fork_version"])
                domain = ssz.compute_domain(ssz.DOMAIN_APPLICATION_BUILDER, fork)
                root = ssz.validator_registration_root(_b(m["fee_recipient"]), int(m["gas_limit"]),
                                                       int(m["timestamp"]), _b(m["pubkey"]))
                ent["registration"] = {"msg": ssz.signing_root(root, domain).hex(),
                                       "sig": _b(br["signature"]).hex()}
            vals.append(ent)
        out.append({"source": f"cluster/examples/cluster-lock-00{i}.json", "threshold": dfn["threshold"],
                    "lock_hash": _b(d["lock_hash"]).hex(), "signature_aggregate": _b(d["signature_aggregate"]).hex(),
                    "validators": vals})
    return out


def attestation_data_kat():
    raw = open(os.path.join(REF, "core/testdata/TestSSZSerialisation_AttestationData.ssz.golden"), "rb").read()
    js = json.load(open(os.path.join(REF, "core/testdata/TestJSONSerialisation_AttestationData.json.golden")))
    ad = js["attestation_data"]
    off = int.from_bytes(raw[0:4], "little")  # core.AttestationData{Data, Duty}: offset of Data
    data = raw[off:off + ssz.ATTESTATION_DATA_SSZ_LEN]
    slot, index, bbr, (se, sr), (te, tr) = ssz.parse_attestation_data(data)
    assert (slot, index) == (int(ad["slot"]), int(ad["index"]))
    assert bbr == _b(ad["beacon_block_root"])
    assert (se, sr) == (int(ad["source"]["epoch"]), _b(ad["source"]["root"]))
    assert (te, tr) == (int(ad["target"]["epoch"]), _b(ad["target"]["root"]))
    return {"ssz": data.hex(), "htr_oracle": ssz.attestation_data_root(data).hex()}


def _td(name):
    return os.path.join(REF, "core/testdata", name)


def duty_roots_kats():
    """The other duty types' SSZ goldens (core/ssz_test.go, core/testdata), each cross-checked field
    by field against its JSON twin; object roots re-derived with oracle/ssz.py (no reference file
    states them).  kind: hbls_duty_signing_roots's (include/hipbls.h)."""
    out = []
    # SignedAggregateAndProof: {message offset, signature}; message = AggregateAndProof
    raw = open(_td("TestSSZSerialisation_SignedAggregateAndProof.ssz.golden"), "rb").read()
    js = json.load(open(_td("TestJSONSerialisation_SignedAggregateAndProof.json.golden")))["message"]
    m = raw[int.from_bytes(raw[0:4], "little"):]
    assert int.from_bytes(m[0:8], "little") == int(js["aggregator_index"])
    assert m[12:108] == _b(js["selection_proof"])
    att = m[int.from_bytes(m[8:12], "little"):]
    assert att[228:] == _b(js["aggregate"]["aggregation_bits"]) and att[132:228] == _b(js["aggregate"]["signature"])
    ad = js["aggregate"]["data"]
    assert ssz.parse_attestation_data(att[4:132])[:3] == (int(ad["slot"]), int(ad["index"]), _b(ad["beacon_block_root"]))
    out.append({"kind": 1, "name": "SignedAggregateAndProof", "ssz": m.hex(),
                "object_root": ssz.aggregate_and_proof_root(m).hex()})
    # SignedSyncContributionAndProof: message = ContributionAndProof (264 B, fixed)
    raw = open(_td("TestSSZSerialisation_SignedSyncContributionAndProof.ssz.golden"), "rb").read()
    js = json.load(open(_td("TestJSONSerialisation_SignedSyncContributionAndProof.json.golden")))["message"]
    m = raw[:264]
    c = js["contribution"]
    assert int.from_bytes(m[0:8], "little") == int(js["aggregator_index"]) and m[168:264] == _b(js["selection_proof"])
    assert int.from_bytes(m[8:16], "little") == int(c["slot"]) and m[16:48] == _b(c["beacon_block_root"])
    assert int.from_bytes(m[48:56], "little") == int(c["subcommittee_index"])
    assert m[56:72] == _b(c["aggregation_bits"]) and m[72:168] == _b(c["signature"])
    out.append({"kind": 2, "name": "SignedSyncContributionAndProof", "ssz": m.hex(),
                "object_root": ssz.contribution_and_proof_root(m).hex()})
    # SyncContributionAndProof: the selection data of its contribution
    raw = open(_td("TestSSZSerialisation_SyncContributionAndProof.ssz.golden"), "rb").read()
    js = json.load(open(_td("TestJSONSerialisation_SyncContributionAndProof.json.golden")))
    slot, sub = int.from_bytes(raw[8:16], "little"), int.from_bytes(raw[48:56], "little")
    assert (slot, sub) == (int(js["contribution"]["slot"]), int(js["contribution"]["subcommittee_index"]))
    sel = slot.to_bytes(8, "little") + sub.to_bytes(8, "little")
    out.append({"kind": 3, "name": "SyncContributionAndProof", "ssz": sel.hex(),
                "object_root": ssz.sync_selection_root(slot, sub).hex()})
    # SyncCommitteeSelection (JSON only): the same selection data
    js = json.load(open(_td("TestJSONSerialisation_SyncCommitteeSelection.json.golden")))
    slot, sub = int(js["slot"]), int(js["subcommittee_index"])
    out.append({"kind": 3, "name": "SyncCommitteeSelection",
                "ssz": (slot.to_bytes(8, "little") + sub.to_bytes(8, "little")).hex(),
                "object_root": ssz.sync_selection_root(slot, sub).hex()})
    # BeaconCommitteeSelection (JSON only): SlotHashRoot(slot)
    js = json.load(open(_td("TestJSONSerialisation_BeaconCommitteeSelection.json.golden")))
    slot = int(js["slot"])
    out.append({"kind": 4, "name": "BeaconCommitteeSelection", "ssz": slot.to_bytes(8, "little").hex(),
                "object_root": ssz.slot_root(slot).hex()})
    # SignedSyncMessage: {slot, beacon_block_root, validator_index, signature}; root = block root
    raw = open(_td("TestSSZSerialisation_SignedSyncMessage.ssz.golden"), "rb").read()
    js = json.load(open(_td("TestJSONSerialisation_SignedSyncMessage.json.golden")))
    assert int.from_bytes(raw[0:8], "little") == int(js["slot"]) and raw[8:40] == _b(js["beacon_block_root"])
    out.append({"kind": 5, "name": "SignedSyncMessage", "ssz": raw[8:40].hex(), "object_root": raw[8:40].hex()})
    # VersionedSignedValidatorRegistration: the teku registration of eth2util/signing/signing_test.go
    # (its signature over this object's signing root is the registration KAT)
    reg = registration_kat_message()
    out.append({"kind": 6, "name": "VersionedSignedValidatorRegistration", "ssz": reg.hex(),
                "object_root": ssz.validator_registration_ssz_root(reg).hex()})
    # SignedVoluntaryExit: {message = VoluntaryExit{epoch, validator_index}, signature}
    raw = open(_td("TestSSZSerialisation_SignedVoluntaryExit.ssz.golden"), "rb").read()
    js = json.load(open(_td("TestJSONSerialisation_SignedVoluntaryExit.json.golden")))
    assert len(raw) == 112 and raw[16:] == _b(js["signature"])
    assert int.from_bytes(raw[0:8], "little") == int(js["message"]["epoch"])
    assert int.from_bytes(raw[8:16], "little") == int(js["message"]["validator_index"])
    out.append({"kind": 7, "name": "SignedVoluntaryExit", "ssz": raw[:16].hex(),
                "object_root": ssz.voluntary_exit_root(raw[:16]).hex()})
    # SignedRandao (JSON only): eth2util.SignedEpoch{epoch, signature}, root = the epoch's chunk
    js = json.load(open(_td("TestJSONSerialisation_SignedRandao.json.golden")))
    ep = int(js["epoch"])
    out.append({"kind": 8, "name": "SignedRandao", "ssz": ep.to_bytes(8, "little").hex(),
                "object_root": ssz.epoch_root(ep).hex()})
    return out


def registration_kat_message() -> bytes:
    """The teku registration message of signing_test.go as its 84-byte SSZ encoding."""
    src = open(os.path.join(REF, "eth2util/signing/signing_test.go")).read()
    fee = bytes.fromhex(re.search(r'"fee_recipient": "0x([0-9a-fA-F]{40})"', src).group(1))
    gas = int(re.search(r'"gas_limit": "(\d+)"', src).group(1))
    ts = int(re.search(r'"timestamp": "(\d+)"', src).group(1))
    pk = bytes.fromhex(re.search(r'"pubkey": "0x([0-9a-f]{96})"', src).group(1))
    return fee + gas.to_bytes(8, "little") + ts.to_bytes(8, "little") + pk


def main():
    kats = {"registration": registration_kat(), "deposit": deposit_kats(), "locks": lock_kats(),
            "attestation_data": attestation_data_kat(), "duty_roots": duty_roots_kats()}
    with open(os.path.join(HERE, "kat_reference.json"), "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote", os.path.join(HERE, "kat_reference.json"))


if __name__ == "__main__":
    main()
