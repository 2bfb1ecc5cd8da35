"""Key-block derivation (CPU, pinned by the reference's PRF vectors) and the
config-1 loopback harness: a client/server pair over a real socket exchanging
Test 22/23-shaped traffic (tests/tlstest.py:66-78, :355-381) with every record
sealed/opened by the gfx950 kernels (GPU)."""
import socket
import threading

import pytest

from tests.golden_io import case_keys


def test_key_block_matches_reference(golden):
    from tlslite_amd.connection import key_block, master_secret
    n = 0
    for c in golden:
        if c["kind"] != "keys":
            continue
        v = tuple(c["version"])
        ms = master_secret(v, bytes.fromhex(c["premaster"]), bytes.fromhex(c["client_random"]),
                           bytes.fromhex(c["server_random"]))
        assert ms.hex() == c["master"], c["name"]
        kb, _ = key_block(v, c["suite"], ms, bytes.fromhex(c["client_random"]), bytes.fromhex(c["server_random"]))
        assert kb.hex() == c["key_block"], c["name"]
        n += 1
    assert n >= 15


def _pair(suite, version):
    from tlslite_amd.connection import RecordLayer, master_secret, pending_states
    pms, cr, sr = bytes(range(48)), bytes(range(32)), bytes(range(32, 64))
    ms = master_secret(version, pms, cr, sr)
    a, b = socket.socketpair()
    cw, crd = pending_states(version, suite, ms, cr, sr, client=True)
    sw, srd = pending_states(version, suite, ms, cr, sr, client=False)
    return RecordLayer(a, version, cw, crd), RecordLayer(b, version, sw, srd), a, b


@pytest.mark.gpu
@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 1)), ("AES256-SHA", (3, 1)), ("RC4-SHA", (3, 1)),
                                           ("AES128-SHA256", (3, 3)), ("3DES-SHA", (3, 2)),
                                           ("RC4-MD5", (3, 0)), ("AES128-SHA", (3, 0))])
def test_loopback_echo(suite, version):
    import os
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible")
    client, server, a, b = _pair(suite, version)
    msgs = [os.urandom(n) for n in (1, 10, 100, 1000)] + [b"hello" * 10000]

    def serve():
        for m in msgs:
            server.write(server.read(min=len(m), max=len(m)))

    t = threading.Thread(target=serve)
    t.start()
    try:
        for m in msgs:
            client.write(m)
            assert client.read(min=len(m), max=len(m)) == m
    finally:
        t.join(timeout=60)
        a.close()
        b.close()
    assert not t.is_alive()
