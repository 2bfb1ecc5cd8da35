"""Batched TLS record seal on the GPU -- the drop-in for the seal block of
tlslite's `TLSRecordLayer._sendMsg` (tlslite/tlsrecordlayer.py:538-617) and
the fragmentation of `writeAsync` (:257-295).

Two levels:
  * `seal(states, records)`      host buffers in, wire bytes out (copies to HBM,
                                 one kernel launch per suite variant, copies back)
  * `seal_dev(...)`              device-resident arenas, no copies: the
                                 throughput path used by bench.py
"""
import ctypes
from collections import OrderedDict

import numpy as np

from . import _native as N
from .constants import ContentType
from .device import DeviceBuffer, synchronize
from .state import STATE_BYTES, pack_states, unpack_states

PT_ALIGN = 16
WIRE_BODY_ALIGN = 16  # record bodies start 16-byte aligned: wire_off % 16 == 11
MAX_FRAGMENT = 16384  # tlsrecordlayer.py:273
MAX_RECORD_BODY = 18432  # tlsrecordlayer.py:871 (16384 + 2048): record_overflow above


class RecordOverflow(ValueError):
    """A record header announced more than 18432 body bytes (record_overflow)."""


class RecordSyntaxError(SyntaxError):
    """Received bytes do not start a TLS record: the first header byte is no content type
    (tlsrecordlayer.py:850-857 raises SyntaxError)."""


class RecordAbruptClose(ConnectionError):
    """A record header announced an empty body: the reference's body loop calls
    sock.recv(0), gets b"" and raises TLSAbruptCloseError (tlsrecordlayer.py:877-889)."""


class BadRecordMAC(ValueError):
    """bad_record_mac alert (tlsrecordlayer.py:1039-1042)."""


class DecryptionFailed(ValueError):
    """decryption_failed alert (tlsrecordlayer.py:964-977)."""


def parse_records(data):
    """Split a received byte stream into (content_type, (major, minor), body)
    records, RecordHeader3.parse style (messages.py:44-49).  Returns
    (records, leftover_bytes) -- an incomplete trailing record stays in the
    leftover."""
    out = []
    pos = 0
    data = bytes(data)
    while pos < len(data):
        if data[pos] not in (20, 21, 22, 23):  # ContentType.all, checked as the byte arrives
            raise RecordSyntaxError("record type byte %d" % data[pos])
        if len(data) - pos < 5:
            break
        ctype, vmaj, vmin = data[pos], data[pos + 1], data[pos + 2]
        length = (data[pos + 3] << 8) | data[pos + 4]
        if length > MAX_RECORD_BODY:
            raise RecordOverflow("record length %d > %d" % (length, MAX_RECORD_BODY))
        if length == 0:
            raise RecordAbruptClose("empty record body (recv(0) in the reference)")
        if len(data) - pos - 5 < length:
            break
        out.append((ctype, (vmaj, vmin), data[pos + 5:pos + 5 + length]))
        pos += 5 + length
    return out, data[pos:]


def plan_write(data, version, block_cipher, max_fragment=MAX_FRAGMENT):
    """Split one write() into record payloads exactly as writeAsync does
    (tlsrecordlayer.py:257-295), including the TLS<=1.0 block-cipher 1/n-1
    split of the first fragment (:543-550).  Empty payloads are dropped: the
    reference emits nothing for them (:551-556)."""
    out = []
    first = True
    for s in range(0, len(data), max_fragment):
        chunk = bytes(data[s:s + max_fragment])
        if first and tuple(version) <= (3, 1) and block_cipher:
            out.append(chunk[:1])
            chunk = chunk[1:]
        if chunk:
            out.append(chunk)
        first = False
    return out


def wire_offsets(wire_lens):
    """Slot layout for a wire arena: each record's 5-byte header at
    off % 16 == 11 so that its body is 16-byte aligned."""
    offs = np.zeros(len(wire_lens), dtype=np.uint64)
    pos = 11
    for i, n in enumerate(wire_lens):
        offs[i] = pos
        pos += int(n)
        pos += (11 - pos) % WIRE_BODY_ALIGN
    return offs, pos


def make_records(pt_off, wire_off, pt_len, content_type=ContentType.application_data, flags=0):
    n = len(pt_len)
    recs = (N.Record * n)()
    a = np.frombuffer(recs, dtype=np.uint8).reshape(n, 24)
    a[:, 0:8] = np.asarray(pt_off, dtype=np.uint64).reshape(n, 1).view(np.uint8)
    a[:, 8:16] = np.asarray(wire_off, dtype=np.uint64).reshape(n, 1).view(np.uint8)
    a[:, 16:20] = np.asarray(pt_len, dtype=np.uint32).reshape(n, 1).view(np.uint8)
    a[:, 20] = np.broadcast_to(np.asarray(content_type, dtype=np.uint8), (n,))
    a[:, 21] = np.broadcast_to(np.asarray(flags, dtype=np.uint8), (n,))
    a[:, 22:24] = 0
    return recs


def make_chains(state_idx, first, count, flags=0):
    n = len(state_idx)
    ch = (N.Chain * n)()
    a = np.frombuffer(ch, dtype=np.uint32).reshape(n, 4)
    a[:, 0] = state_idx
    a[:, 1] = first
    a[:, 2] = count
    a[:, 3] = flags
    return ch


def seal_workspace_bytes(nrecords):
    return int(N.lib.tlsgpu_seal_workspace_bytes(int(nrecords)))


def seal_cipher_kernel(variant, nchains):
    """The cipher-phase kernel (rocprofv3 name stem) a seal call of `nchains` chains of
    `variant` runs on the current device: the library picks the layout from the chains
    per CU (tlsgpu_seal_cipher_kernel)."""
    buf = ctypes.create_string_buffer(96)
    N.call("tlsgpu_seal_cipher_kernel", int(variant), int(nchains), buf, len(buf))
    return buf.value.decode()


def _p(x):
    return x.ptr if isinstance(x, DeviceBuffer) else ctypes.c_void_p(x)


def _size(x, given, what):
    """An arena's byte size for the ABI-6 bounds: given explicitly, or the DeviceBuffer's."""
    if given is not None:
        return int(given)
    if isinstance(x, DeviceBuffer):
        return int(x.nbytes)
    raise ValueError("%s is a raw address: pass its size (the library checks every record against it)" % what)


def _nstates(states, nstates):
    if nstates is not None:
        return int(nstates)
    if isinstance(states, DeviceBuffer):
        return int(states.nbytes // STATE_BYTES)
    raise ValueError("states is a raw address: pass nstates")


def seal_dev(chains, nchains, records, nrecords, pt, wire, states, wire_len, variant, workspace=None, stream=None,
             pt_bytes=None, wire_bytes=None, nstates=None):
    """Device-resident batch seal (all pointers are DeviceBuffer / addresses).
    workspace: DeviceBuffer of >= seal_workspace_bytes(nrecords), or None for
    the library-owned one (one per stream).  pt_bytes / wire_bytes / nstates: the
    arenas' sizes and the state count (ABI 6 bounds; taken from DeviceBuffers when not
    given): a record outside them gets wire_len = EINVAL and is not sealed."""
    N.call("tlsgpu_seal_dev", _p(chains), nchains, _p(records), int(nrecords), _p(pt), _size(pt, pt_bytes, "pt"),
           _p(wire), _size(wire, wire_bytes, "wire"), _p(states), _nstates(states, nstates), _p(wire_len),
           variant, None if workspace is None else _p(workspace), 0 if workspace is None else workspace.nbytes,
           stream.handle if stream is not None else None)


class SealPipeline:
    """Overlapped batch seal (tlsgpu_pipeline_*): the per-record MAC phase of
    call k+1 runs while the CBC phase of call k is still encrypting, on two
    library-owned streams with double-buffered workspaces.  Each call has the
    semantics of seal_dev; results are complete after synchronize()."""

    def __init__(self, max_records):
        h = ctypes.c_void_p()
        N.call("tlsgpu_pipeline_create", ctypes.byref(h), int(max_records))
        self.handle = h
        self.max_records = int(max_records)

    def seal(self, chains, nchains, records, nrecords, pt, wire, states, wire_len, variant,
             cipher_start=None, cipher_stop=None, pt_bytes=None, wire_bytes=None, nstates=None):
        N.call("tlsgpu_pipeline_seal", self.handle, _p(chains), nchains, _p(records), int(nrecords), _p(pt),
               _size(pt, pt_bytes, "pt"), _p(wire), _size(wire, wire_bytes, "wire"), _p(states),
               _nstates(states, nstates), _p(wire_len), variant,
               cipher_start.handle if cipher_start is not None else None,
               cipher_stop.handle if cipher_stop is not None else None)

    def synchronize(self):
        N.call("tlsgpu_pipeline_synchronize", self.handle)

    def close(self):
        if self.handle is not None and self.handle.value:
            N.call("tlsgpu_pipeline_destroy", self.handle)
        self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class HostSealPipeline:
    """Seal and open batches whose arenas live in HOST memory (tlsgpu_host_pipeline_*):
    seal -- the records' socket-buffer hand-off (tlsrecordlayer.py:616-620) with H2D copy,
    seal and D2H copy of successive sub-batches overlapped on `depth` streams; open -- the
    receive path from socket buffers (:832-893, :958-1044): H2D copy, framing and open on the
    device, D2H copy of the plaintext.  Pinned host arrays (device.PinnedBuffer) are copied
    directly, pageable ones through library-owned pinned staging buffers."""

    def __init__(self, chunk_bytes=64 << 20, depth=3):
        h = ctypes.c_void_p()
        N.call("tlsgpu_host_pipeline_create", ctypes.byref(h), int(chunk_bytes), int(depth))
        self.handle = h

    def seal(self, chains, records, pt_host, wire_host, states, wire_len_host, variant, nstates=None):
        """chains / records: ctypes arrays (host); pt_host / wire_host: numpy uint8
        arrays (host); states: DeviceBuffer; wire_len_host: numpy int32 [nrecords]."""
        N.call("tlsgpu_host_pipeline_seal", self.handle, ctypes.addressof(chains), len(chains),
               ctypes.addressof(records), len(records), pt_host.ctypes.data_as(ctypes.c_void_p), pt_host.nbytes,
               wire_host.ctypes.data_as(ctypes.c_void_p), wire_host.nbytes, states.ptr, _nstates(states, nstates),
               wire_len_host.ctypes.data_as(ctypes.c_void_p), variant)

    def open(self, rx_host, spans, pt_host, states, variant, max_records=None, chain_flags=None, nstates=None,
             out=None):
        """Open the records in connections' received bytes (tlsgpu_host_pipeline_open).
        rx_host: numpy uint8 (host) holding every connection's bytes; spans: ctypes array of
        N.Span {off, len, state}; pt_host: numpy uint8 (host, >= rx_host.nbytes) for the
        opened bodies; states: DeviceBuffer of read states.  max_records None: every record
        the bytes can hold.  out: optional dict of preallocated host arrays (records /
        status: pinned ones are copied to directly).  Returns a dict: records (ctypes
        N.OpenRecord array), status (int32), chains (N.Chain array), consumed (uint32),
        frame_status (int32), total."""
        n = len(spans)
        flags = N.CHAIN_STOP_ON_ALERT if chain_flags is None else int(chain_flags)
        if max_records is None:
            max_records = sum(int(sp.len) // 5 for sp in spans) + 1
        out = dict(out or {})
        recs = out.get("records")
        if recs is None:
            recs = (N.OpenRecord * max(1, max_records))()
        status = out.get("status")
        if status is None:
            status = np.zeros(max(1, max_records), dtype=np.int32)
        chains = (N.Chain * n)()
        consumed = np.zeros(n, dtype=np.uint32)
        fstatus = np.zeros(n, dtype=np.int32)
        total = ctypes.c_uint32()
        rp = recs.ctypes.data_as(ctypes.c_void_p) if isinstance(recs, np.ndarray) else ctypes.addressof(recs)
        N.call("tlsgpu_host_pipeline_open", self.handle, rx_host.ctypes.data_as(ctypes.c_void_p), rx_host.nbytes,
               ctypes.addressof(spans), n, flags, pt_host.ctypes.data_as(ctypes.c_void_p), pt_host.nbytes,
               states.ptr, _nstates(states, nstates), variant, rp, int(max_records), ctypes.addressof(chains),
               consumed.ctypes.data_as(ctypes.c_void_p), fstatus.ctypes.data_as(ctypes.c_void_p),
               status.ctypes.data_as(ctypes.c_void_p), ctypes.byref(total))
        return {"records": recs, "status": status[: total.value], "chains": chains, "consumed": consumed,
                "frame_status": fstatus, "total": total.value}

    @property
    def d2h_path(self):
        """How the pipeline's large D2H copies run: None (not chosen yet), "engine" (the copy
        engine) or "stores" (the GPU's own stores into the pinned destination)."""
        v = ctypes.c_int()
        N.call("tlsgpu_host_pipeline_d2h_path", self.handle, ctypes.byref(v))
        return {-1: None, 0: "engine", 1: "stores"}[v.value]

    def close(self):
        if self.handle is not None and self.handle.value:
            N.call("tlsgpu_host_pipeline_destroy", self.handle)
        self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def seal(states, records, stream=None, pt_shift=0, wire_shift=0):
    """Seal records on the GPU.

    states:  list of ConnectionState (updated in place: seqnum, CBC residue, RC4)
    records: list of (state_index, payload, content_type=23, flags=0); records
             of one state are sealed in list order, like successive _sendMsg calls.
    Returns the list of wire records (b"" for an empty payload).
    pt_shift / wire_shift (tests): place every record's plaintext at
    pt_off % 16 == pt_shift and its body at (wire_off + 5) % 16 == wire_shift
    instead of the 16-byte grid, to exercise the kernels' unaligned paths.
    """
    norm = []
    for r in records:
        si, payload = r[0], bytes(r[1])
        ct = r[2] if len(r) > 2 else ContentType.application_data
        fl = r[3] if len(r) > 3 else 0
        norm.append((si, payload, ct, fl))
    nrec = len(norm)
    if nrec == 0:
        return []
    by_state = OrderedDict()
    for i, (si, _, _, _) in enumerate(norm):
        by_state.setdefault(si, []).append(i)
    # descriptor order: chains contiguous
    order = [i for idxs in by_state.values() for i in idxs]
    pos_of = {i: k for k, i in enumerate(order)}
    wlen = []
    for i in order:
        si, payload, _, _ = norm[i]
        n = len(payload)
        try:
            wlen.append(states[si].wire_len(n))
        except N.TLSGPUError as e:
            if e.code == N.ETOOBIG:
                raise ValueError("Can't represent value in specified length")  # codec.py:19-20
            raise
    pt_off = np.zeros(nrec, dtype=np.uint64)
    pos = 0
    for k, i in enumerate(order):
        pt_off[k] = pos + pt_shift
        pos += len(norm[i][1])
        pos += (-pos) % PT_ALIGN
    pt_total = max(pos, 16) + pt_shift
    wire_off, wire_total = wire_offsets(wlen)
    wire_off += np.uint64(wire_shift)
    wire_total += wire_shift
    pt_host = np.zeros(pt_total, dtype=np.uint8)
    for k, i in enumerate(order):
        b = norm[i][1]
        if b:
            pt_host[int(pt_off[k]):int(pt_off[k]) + len(b)] = np.frombuffer(b, dtype=np.uint8)
    recs = make_records(pt_off, wire_off, [len(norm[i][1]) for i in order], [norm[i][2] for i in order],
                        [norm[i][3] for i in order])
    # chains, bucketed by variant
    sidx = list(by_state.keys())
    buckets = OrderedDict()
    first = 0
    for si in sidx:
        cnt = len(by_state[si])
        buckets.setdefault(states[si].variant, []).append((si, first, cnt))
        first += cnt
    d_pt = DeviceBuffer(pt_total)
    d_wire = DeviceBuffer(wire_total)
    d_recs = DeviceBuffer(ctypes.sizeof(recs))
    d_len = DeviceBuffer(4 * nrec)
    d_states = DeviceBuffer(STATE_BYTES * len(states))
    d_pt.upload(pt_host, stream=stream)
    d_recs.upload(np.frombuffer(recs, dtype=np.uint8), stream=stream)
    d_states.upload(pack_states(states), stream=stream)
    d_wire.zero(stream)
    chain_bufs = []
    for var, chs in buckets.items():
        c = make_chains([x[0] for x in chs], [x[1] for x in chs], [x[2] for x in chs])
        d_ch = DeviceBuffer(ctypes.sizeof(c))
        d_ch.upload(np.frombuffer(c, dtype=np.uint8), stream=stream)
        chain_bufs.append(d_ch)
        seal_dev(d_ch, len(chs), d_recs, nrec, d_pt, d_wire, d_states, d_len, var, None, stream)
    if stream is not None:
        stream.synchronize()
    wire_host = d_wire.download()
    lens = d_len.download().view(np.int32)
    unpack_states(d_states.download(), states)
    synchronize()
    out = [b""] * nrec
    for k, i in enumerate(order):
        L = int(lens[k])
        if L < 0:
            raise N.TLSGPUError(L, "seal record %d" % i)
        if L != wlen[k]:
            raise RuntimeError("wire length mismatch %d != %d" % (L, wlen[k]))
        o = int(wire_off[k])
        out[i] = wire_host[o:o + L].tobytes()
    return out


def make_open_records(ct_off, pt_off, ct_len, content_type):
    n = len(ct_len)
    recs = (N.OpenRecord * n)()
    a = np.frombuffer(recs, dtype=np.uint8).reshape(n, 24)
    a[:, 0:8] = np.asarray(ct_off, dtype=np.uint64).reshape(n, 1).view(np.uint8)
    a[:, 8:16] = np.asarray(pt_off, dtype=np.uint64).reshape(n, 1).view(np.uint8)
    a[:, 16:20] = np.asarray(ct_len, dtype=np.uint32).reshape(n, 1).view(np.uint8)
    a[:, 20] = np.broadcast_to(np.asarray(content_type, dtype=np.uint8), (n,))
    a[:, 21:24] = 0
    return recs


def open_workspace_bytes(nrecords):
    return int(N.lib.tlsgpu_open_workspace_bytes(int(nrecords)))


def open_dev(chains, nchains, records, nrecords, wire, pt, states, status, variant, workspace=None, stream=None,
             wire_bytes=None, pt_bytes=None, nstates=None):
    """Device-resident batch open (decrypt + padding + MAC check).  workspace:
    DeviceBuffer of >= open_workspace_bytes(nrecords), or None (library-owned).
    wire_bytes / pt_bytes / nstates: ABI 6 bounds (from DeviceBuffers when not given)."""
    N.call("tlsgpu_open_dev", _p(chains), nchains, _p(records), int(nrecords), _p(wire), _size(wire, wire_bytes, "wire"),
           _p(pt), _size(pt, pt_bytes, "pt"), _p(states), _nstates(states, nstates), _p(status),
           variant, None if workspace is None else _p(workspace), 0 if workspace is None else workspace.nbytes,
           stream.handle if stream is not None else None)


def set_open_parts(mode=N.OPEN_SPLIT_AUTO, min_records=0):
    """How CBC-suite opens are split (process-wide): N.OPEN_SPLIT_AUTO (the library picks),
    N.OPEN_SPLIT_CHAINS (chain-range parts for every batch of >= min_records records: tests
    run the form on small batches), N.OPEN_SPLIT_NONE (one pass each), N.OPEN_SPLIT_BLOCKS
    (3DES: block-range parts for every batch of >= min_records records)."""
    N.call("tlsgpu_set_open_parts", int(mode), int(min_records))


def open_records(states, records, stream=None, stop_on_alert=True):
    """Open (decrypt + verify) records on the GPU -- the batched counterpart of
    _decryptRecord (tlsrecordlayer.py:958-1044).

    states:  list of read-direction ConnectionState (updated in place)
    records: list of (state_index, content_type, body); records of one state
             are opened in list order.
    stop_on_alert: a connection stops at its first alert, as the reference's
             does (_getMsg raises, _sendError closes it, :1039-1042): later
             records of that state come back as N.ALERT_SKIPPED and the state is
             left as the failing record left it.  False opens every record, as
             successive bare _decryptRecord calls would.
    Returns a list of (status, plaintext): status 0 and the plaintext bytes,
    or an alert code (N.ALERT_BAD_RECORD_MAC / N.ALERT_DECRYPTION_FAILED /
    N.ALERT_SKIPPED) and None.
    """
    nrec = len(records)
    if nrec == 0:
        return []
    d_states = DeviceBuffer(STATE_BYTES * len(states))
    d_states.upload(pack_states(states), stream=stream)
    b = _OpenBatch(states, records, stream, stop_on_alert)
    for var, d_ch, nch in b.calls:
        open_dev(d_ch, nch, b.d_recs, nrec, b.d_ct, b.d_pt, d_states, b.d_st, var, stream=stream)
    if stream is not None:
        stream.synchronize()
    out = b.results()
    unpack_states(d_states.download(), states)
    synchronize()
    return out


class _OpenBatch:
    """One batch of received records staged in device memory for an open: the ciphertext
    arena (records of one state contiguous, in list order), the plaintext arena, descriptors,
    status, and one chain list per suite variant (self.calls: (variant, chains, nchains))."""

    def __init__(self, states, records, stream, stop_on_alert):
        self.nrec = nrec = len(records)
        by_state = OrderedDict()
        for i, r in enumerate(records):
            by_state.setdefault(r[0], []).append(i)
        self.order = order = [i for idxs in by_state.values() for i in idxs]
        self.ct_off = ct_off = np.zeros(nrec, dtype=np.uint64)
        pos = 0
        for k, i in enumerate(order):
            ct_off[k] = pos
            pos += len(records[i][2])
            pos += (-pos) % PT_ALIGN
        total = max(pos, 16)
        host = np.zeros(total, dtype=np.uint8)
        for k, i in enumerate(order):
            b = bytes(records[i][2])
            if b:
                host[int(ct_off[k]):int(ct_off[k]) + len(b)] = np.frombuffer(b, dtype=np.uint8)
        recs = make_open_records(ct_off, ct_off, [len(records[i][2]) for i in order],
                                 [records[i][1] for i in order])
        buckets = OrderedDict()
        first = 0
        for si, idxs in by_state.items():
            buckets.setdefault(states[si].variant, []).append((si, first, len(idxs)))
            first += len(idxs)
        self.d_ct = DeviceBuffer(total)
        self.d_pt = DeviceBuffer(total)
        self.d_recs = DeviceBuffer(ctypes.sizeof(recs))
        self.d_st = DeviceBuffer(4 * nrec)
        self.d_ct.upload(host, stream=stream)
        self.d_recs.upload(np.frombuffer(recs, dtype=np.uint8), stream=stream)
        self.d_pt.zero(stream)
        self.calls = []
        for var, chs in buckets.items():
            c = make_chains([x[0] for x in chs], [x[1] for x in chs], [x[2] for x in chs],
                            N.CHAIN_STOP_ON_ALERT if stop_on_alert else 0)
            d_ch = DeviceBuffer(ctypes.sizeof(c))
            d_ch.upload(np.frombuffer(c, dtype=np.uint8), stream=stream)
            self.calls.append((var, d_ch, len(chs)))

    def results(self):
        """[(status, plaintext or None)] in the batch's list order (after the open completed)."""
        pt_host = self.d_pt.download()
        status = self.d_st.download().view(np.int32)
        out = [None] * self.nrec
        for k, i in enumerate(self.order):
            st = int(status[k])
            if st < 0:
                out[i] = (st, None)
            else:
                o = int(self.ct_off[k])
                out[i] = (0, pt_host[o:o + st].tobytes())
        return out


def open_batches(states, batches, stream=None, stop_on_alert=True):
    """Open successive batches of received records with the states device-resident
    throughout (one open_dev call per batch and suite variant, in order on one stream) --
    what open_records on each batch in turn returns, with the connection semantics carried
    across batches: a connection stopped by an alert in one batch is closed in its state
    (ConnState.closed) and reports N.ALERT_SKIPPED in later ones.  batches: lists as
    open_records takes them.  Returns one result list per batch."""
    batches = [list(b) for b in batches]
    d_states = DeviceBuffer(STATE_BYTES * len(states))
    d_states.upload(pack_states(states), stream=stream)
    staged = []
    for recs in batches:
        b = _OpenBatch(states, recs, stream, stop_on_alert) if recs else None
        if b is not None:
            for var, d_ch, nch in b.calls:
                open_dev(d_ch, nch, b.d_recs, b.nrec, b.d_ct, b.d_pt, d_states, b.d_st, var, stream=stream)
        staged.append(b)
    if stream is not None:
        stream.synchronize()
    out = [b.results() if b is not None else [] for b in staged]
    unpack_states(d_states.download(), states)
    synchronize()
    return out


def frame_workspace_bytes(n):
    return int(N.lib.tlsgpu_frame_workspace_bytes(int(n)))


def frame_dev(stream, conns, n, records, max_records, chains, consumed, status, total, workspace=None,
              chain_flags=None, s=None, stream_bytes=None):
    """Receive framing on the device (tlsgpu_frame_dev): n connections' received bytes in the
    `stream` arena (conns: tlsgpu_span {off, len, state} per connection) -> open descriptors
    (records, from 0, in connection order), one chain per connection, consumed bytes and a
    status per connection, the record total in `total` (one uint32).  All DeviceBuffers;
    workspace None: a temporary one."""
    ws = workspace if workspace is not None else DeviceBuffer(max(16, frame_workspace_bytes(n)))
    flags = N.CHAIN_STOP_ON_ALERT if chain_flags is None else int(chain_flags)
    N.call("tlsgpu_frame_dev", _p(stream), _size(stream, stream_bytes, "stream"), _p(conns), int(n), _p(records),
           int(max_records), _p(chains), flags, _p(consumed), _p(status), _p(total), _p(ws), ws.nbytes,
           s.handle if s is not None else None)
    return ws


def frame_streams(streams, max_records=None):
    """Frame each connection's received bytes on the GPU (frame_dev) and bring the result back:
    one (status, consumed, [(content_type, body bytes), ...]) per connection.  Test / host
    convenience: the device-resident path feeds frame_dev's descriptors to open_dev."""
    n = len(streams)
    offs, pos = [], 0
    for b in streams:
        offs.append(pos)
        pos += len(b)
        pos += (-pos) % PT_ALIGN
    arena = np.zeros(max(pos, 16), dtype=np.uint8)
    for o, b in zip(offs, streams):
        if b:
            arena[o:o + len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
    spans = (N.Span * n)()
    a = np.frombuffer(spans, dtype=np.uint8).reshape(n, 16)
    a[:, 0:8] = np.asarray(offs, dtype=np.uint64).reshape(n, 1).view(np.uint8)
    a[:, 8:12] = np.asarray([len(b) for b in streams], dtype=np.uint32).reshape(n, 1).view(np.uint8)
    a[:, 12:16] = np.arange(n, dtype=np.uint32).reshape(n, 1).view(np.uint8)
    maxr = sum(len(b) // 5 + 1 for b in streams) if max_records is None else int(max_records)
    d_s, d_sp = DeviceBuffer(arena.nbytes), DeviceBuffer(ctypes.sizeof(spans))
    d_s.upload(arena)
    d_sp.upload(np.frombuffer(spans, dtype=np.uint8))
    d_r = DeviceBuffer(max(1, maxr) * ctypes.sizeof(N.OpenRecord))
    d_c, d_cons, d_st, d_tot = (DeviceBuffer(16 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(16))
    frame_dev(d_s, d_sp, n, d_r, maxr, d_c, d_cons, d_st, d_tot)
    synchronize()
    total = int(d_tot.download()[:4].view(np.uint32)[0])
    recs = np.frombuffer(d_r.download(), dtype=np.uint8).reshape(-1, ctypes.sizeof(N.OpenRecord))
    ch = d_c.download().view(np.uint32).reshape(n, 4)
    cons = d_cons.download().view(np.uint32)
    st = d_st.download().view(np.int32)
    out = []
    for i in range(n):
        first, count = int(ch[i, 1]), int(ch[i, 2])
        rs = []
        for r in recs[first:first + count]:
            off = int(r[0:8].view(np.uint64)[0])
            ln = int(r[16:20].view(np.uint32)[0])
            rs.append((int(r[20]), arena[off:off + ln].tobytes()))
        out.append((int(st[i]), int(cons[i]), rs))
    return out, total


def open_stream(state, data):
    """Parse + open every complete record of one connection's byte stream.
    Raises BadRecordMAC / DecryptionFailed like the reference's alerts."""
    recs, rest = parse_records(data)
    res = open_records([state], [(0, ct, body) for ct, _, body in recs])
    out = []
    for (ct, _, _), (st, p) in zip(recs, res):
        if st == N.ALERT_BAD_RECORD_MAC:
            raise BadRecordMAC("MAC failure (or padding failure)")
        if st == N.ALERT_DECRYPTION_FAILED:
            raise DecryptionFailed("Encrypted data not a multiple of blocksize")
        out.append((ct, p))
    return out, rest


def seal_write(state, data, content_type=ContentType.application_data, fault=0):
    """One TLSRecordLayer.write(): fragmentation + BEAST split + seal.
    Returns the list of wire records in send order."""
    payloads = plan_write(data, state.version, state.isBlockCipher)
    return seal([state], [(0, p, content_type, fault) for p in payloads])
