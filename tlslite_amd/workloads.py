"""Device-resident synthetic workloads for the BASELINE.json configs
(SURVEY.md §8d).  A workload is plain data (keys, IVs, seqnums, offsets,
plaintext seed) plus the HBM arenas built from it, so the same description
can be replayed by a CPU checker.

  cfg2  64 Ki x 16 KiB records, AES-128-CBC + HMAC-SHA1, TLS 1.2, one key /
        MAC key / fixedIV, per-record CBC IV, seqnum = record index
  cfg3  1 Mi x 1434 B records, AES-256-CBC + HMAC-SHA256, TLS 1.2, per-record IV
  cfg4  C connections x R records, AES-128-CBC-SHA, per-connection keys,
        records chained inside a connection (residue / seqnum carried)
  cfg5  RC4-SHA and 3DES-EDE-CBC-SHA records interleaved 50/50 (seeded
        shuffle), fresh connection per record, one launch per suite variant

Plaintext bytes come from the device splitmix64 generator
(tlsgpu_fill_pattern) with a per-config seed: byte i of the arena is byte
(i & 7) of splitmix64(seed + (i >> 3)).
"""
import ctypes

import numpy as np

from . import _native as N
from .constants import ContentType, suite_primitives
from .device import DeviceBuffer, fill_pattern
from .recordlayer import make_chains, make_open_records, make_records, open_dev, open_workspace_bytes
from .state import STATE_BYTES, ConnectionState


def _round_up(x, a):
    return (x + a - 1) // a * a


class Group:
    """Connections of one suite in a workload."""

    def __init__(self, suite, version, keys, ivs, mac_keys, fixed_ivs, seq0, recs_per_conn, pt_len):
        self.suite, self.version = suite, tuple(version)
        self.keys, self.ivs, self.mac_keys, self.fixed_ivs = keys, ivs, mac_keys, fixed_ivs
        self.seq0 = np.asarray(seq0, dtype=np.uint64)
        self.recs_per_conn, self.pt_len = int(recs_per_conn), int(pt_len)

    @property
    def nconn(self):
        return len(self.seq0)


class Workload:
    """Host description + device arenas.  Record r of the flat descriptor
    array belongs to chain chain_of[r]; chains of one variant are launched
    together."""

    def __init__(self, name, groups, seed, rec_order=None, chain_stream_start=None, rec_ctype=None, rec_flags=None,
                 pt_align=16):
        self.name, self.groups, self.seed = name, groups, seed
        # flat records in chain order
        states, pt_len, chain_first, chain_count, chain_group = [], [], [], [], []
        r = 0
        for gi, g in enumerate(groups):
            for c in range(g.nconn):
                chain_first.append(r)
                chain_count.append(g.recs_per_conn)
                chain_group.append(gi)
                pt_len += [g.pt_len] * g.recs_per_conn
                r += g.recs_per_conn
        self.n_records = r
        self.n_chains = len(chain_first)
        # per-record content type / fault flags (tlsgpu_record), in chain order
        self.rec_ctype = (np.full(r, ContentType.application_data, dtype=np.uint8) if rec_ctype is None
                          else np.asarray(rec_ctype, dtype=np.uint8))
        self.rec_flags = np.zeros(r, dtype=np.uint8) if rec_flags is None else np.asarray(rec_flags, dtype=np.uint8)
        self.pt_len = np.asarray(pt_len, dtype=np.uint32)
        self.chain_first = np.asarray(chain_first, dtype=np.uint32)
        self.chain_count = np.asarray(chain_count, dtype=np.uint32)
        self.chain_group = np.asarray(chain_group, dtype=np.int32)
        # arena placement: rec_order permutes records in memory (cfg5 interleave)
        order = np.arange(r) if rec_order is None else np.asarray(rec_order)
        self.slot_of = np.empty(r, dtype=np.int64)
        self.slot_of[order] = np.arange(r)
        # plaintext slots at pt_align-byte boundaries (16: packed, bench.py's default since round 4,
        # as a TLS stack fills an arena; bench.py --pt-align 128 puts every record on a line, so the
        # MAC kernel's 64-B chunks never straddle two -- round 3's cfg3 figures used that layout)
        self.pt_align = int(pt_align)
        pt_stride = np.array([_round_up(int(x), self.pt_align) for x in self.pt_len])
        wlen = np.array([self._wire_len(g, int(n)) for g, n in self._rec_groups()], dtype=np.int64)
        self.wire_len = wlen
        # offsets in slot order
        ps = pt_stride[order]
        pt_off_slot = np.concatenate([[0], np.cumsum(ps)[:-1]])
        # Wire slots, packed in slot order: each record's body after its explicit IV starts at
        # the same offset modulo 128 B as its plaintext (pt_off is 16-aligned, so the body is
        # too), so the cipher phase's groups, aligned to the output's lines, also load whole
        # plaintext lines (tg_aes3.h pcbc_bulk).  A sender writev()s [wire_off, wire_off+5+C).
        eiv = np.array([self._explicit_iv(g) for g, _ in self._rec_groups()], dtype=np.int64)[order]
        wl_slot = wlen[order]
        wire_off_slot = np.empty(r, dtype=np.int64)
        cur = 16
        for k in range(r):
            target = (int(pt_off_slot[k]) - 5 - int(eiv[k])) % 128
            wo = cur + ((target - cur) % 128)
            wire_off_slot[k] = wo
            cur = wo + int(wl_slot[k])
        self.pt_off = pt_off_slot[self.slot_of].astype(np.uint64)
        self.wire_off = wire_off_slot[self.slot_of].astype(np.uint64)
        self.pt_bytes = int(ps.sum())
        self.wire_bytes = cur + 128
        self.plaintext_total = int(self.pt_len.sum())
        self.wire_total = int(wlen.sum())
        # position of each chain's plaintext in the splitmix stream: by default
        # the arena offset; sharded workloads pass the unsharded (global) one
        # so a connection's bytes do not depend on which rank owns it
        first_off = self.pt_off[self.chain_first] if self.n_chains else np.zeros(0, dtype=np.uint64)
        self.chain_stream_start = (first_off.astype(np.uint64) if chain_stream_start is None
                                   else np.asarray(chain_stream_start, dtype=np.uint64))
        self._contiguous_fill = chain_stream_start is None

    def fill_plan(self):
        """[(arena_offset, nbytes, stream_start)] covering every chain's plaintext."""
        if self._contiguous_fill:
            return [(0, self.pt_bytes, 0)]
        plan = []
        for c in range(self.n_chains):
            a = int(self.chain_first[c])
            b = a + int(self.chain_count[c]) - 1
            off = int(self.pt_off[a])
            end = int(self.pt_off[b]) + int(self.pt_len[b])
            plan.append((off, end - off, int(self.chain_stream_start[c])))
        return plan

    def host_plaintext(self, fill_fn):
        """Host copy of the plaintext arena; fill_fn(n, seed, start) -> uint8 array."""
        out = np.zeros(self.pt_bytes, dtype=np.uint8)
        for off, n, start in self.fill_plan():
            out[off:off + n] = fill_fn(n, self.seed, start)
        return out

    def _rec_groups(self):
        for gi, g in enumerate(self.groups):
            for _ in range(g.nconn * g.recs_per_conn):
                yield g, g.pt_len

    @staticmethod
    def _explicit_iv(g):
        """bytes of explicit IV before the body (TLS >= 1.1 block ciphers, tlsrecordlayer.py:594-595)"""
        cipher = suite_primitives(g.suite)[0]
        if cipher == "rc4":
            return 0
        return (8 if cipher == "3des" else 16) if g.version >= (3, 2) else 0

    @staticmethod
    def _wire_len(g, n):
        cipher, mac, _, _, ml = suite_primitives(g.suite)
        if n == 0:
            return 0
        if cipher == "rc4":
            return 5 + n + ml
        bs = 8 if cipher == "3des" else 16
        e = bs if g.version >= (3, 2) else 0
        cur = e + n + ml
        return 5 + cur + (bs - cur % bs)

    # ------------------------------------------------------------ host states
    def host_states(self):
        """numpy uint8 [n_chains * 2048] of initial connection states."""
        out = np.zeros(self.n_chains * STATE_BYTES, dtype=np.uint8)
        ci = 0
        for g in self.groups:
            proto_cache = {}
            for c in range(g.nconn):
                k = g.keys[c % len(g.keys)]
                mk = g.mac_keys[c % len(g.mac_keys)]
                fiv = g.fixed_ivs[c % len(g.fixed_ivs)] if g.fixed_ivs is not None else None
                key = (bytes(k), bytes(mk), None if fiv is None else bytes(fiv))
                if key not in proto_cache:
                    iv0 = bytes(g.ivs[c]) if g.ivs is not None else b""
                    proto_cache[key] = ConnectionState.for_suite(g.suite, g.version, key[0], iv0, key[1], key[2], 0)
                st = proto_cache[key]
                blob = out[ci * STATE_BYTES:(ci + 1) * STATE_BYTES]
                blob[:] = np.frombuffer(st.raw, dtype=np.uint8)
                p = (ctypes.c_uint8 * STATE_BYTES).from_buffer(blob)
                if g.ivs is not None and len(g.ivs[c]):
                    N.call("tlsgpu_conn_state_set_iv", p, ctypes.c_char_p(bytes(g.ivs[c])), len(g.ivs[c]))
                N.call("tlsgpu_conn_state_set_seqnum", p, int(g.seq0[c]))
                ci += 1
        return out

    # ------------------------------------------------------------ device arenas
    def to_device(self, stream=None, fill=True):
        self.d_pt = DeviceBuffer(self.pt_bytes)
        self.d_wire = DeviceBuffer(self.wire_bytes)
        self.d_len = DeviceBuffer(4 * self.n_records)
        recs = make_records(self.pt_off, self.wire_off, self.pt_len, self.rec_ctype, self.rec_flags)
        self.d_recs = DeviceBuffer(ctypes.sizeof(recs))
        self.d_recs.upload(np.frombuffer(recs, dtype=np.uint8))
        st = self.host_states()
        self.d_states = DeviceBuffer(st.nbytes)
        self.d_states0 = DeviceBuffer(st.nbytes)
        self.d_states0.upload(st)
        self.d_states.upload(st)
        # one chain array per variant
        self.launches = []
        self.launch_alg_bytes = []
        var_of_group = [ConnectionState.for_suite(
            g.suite, g.version, bytes(g.keys[0]), bytes(g.ivs[0]) if g.ivs is not None else b"",
            bytes(g.mac_keys[0]), bytes(g.fixed_ivs[0]) if g.fixed_ivs is not None else None).variant
            for g in self.groups]
        # 3DES (the longest-running variant) first, so that bench.py's cipher events, which
        # bracket the first launch, time the dominant kernel of a mixed batch
        for var in sorted(set(var_of_group), key=lambda v: (0 if (v & 0xff) == N.CIPHER_3DES else 1, v)):
            idx = [c for c in range(self.n_chains) if var_of_group[self.chain_group[c]] == var]
            ch = make_chains(np.asarray(idx, dtype=np.uint32), self.chain_first[idx], self.chain_count[idx])
            d = DeviceBuffer(ctypes.sizeof(ch))
            d.upload(np.frombuffer(ch, dtype=np.uint8))
            self.launches.append((var, d, len(idx)))
            recs = np.concatenate([np.arange(int(self.chain_first[c]), int(self.chain_first[c] + self.chain_count[c]))
                                   for c in idx]) if idx else np.zeros(0, dtype=np.int64)
            # algorithmic bytes of this launch (P read + 5+C written)
            self.launch_alg_bytes.append(int(self.pt_len[recs].astype(np.int64).sum() + self.wire_len[recs].sum()))
        if fill:
            for off, n, start in self.fill_plan():
                fill_pattern(self.d_pt, n, self.seed, start, off, stream)
        self.d_wire.zero(stream)
        return self

    def uses_split_pipeline(self):
        """True when some launch is an AES suite (prefix/MAC/CBC phases that the
        seal pipeline overlaps across calls)."""
        return any((var & 0xff) in (N.CIPHER_AES128, N.CIPHER_AES256) for var, _, _ in self.launches)

    def reset_states(self, stream=None):
        N.call("tlsgpu_memcpy_d2d", self.d_states.ptr, self.d_states0.ptr, self.d_states.nbytes,
               stream.handle if stream else None)

    def launch(self, streams=None, pipeline=None, cipher_events=None):
        """Seal every record once (one seal call per suite variant; with
        several streams the variants run concurrently).  With a SealPipeline
        the calls are queued on it instead (MAC/cipher phases overlap across
        calls); cipher_events=(start, stop) bracket the first call's cipher
        kernel."""
        if pipeline is not None:
            for i, (var, d_ch, nch) in enumerate(self.launches):
                ev = cipher_events if (cipher_events and i == 0) else (None, None)
                pipeline.seal(d_ch, nch, self.d_recs, self.n_records, self.d_pt, self.d_wire, self.d_states,
                              self.d_len, var, ev[0], ev[1])
            return
        if not hasattr(self, "d_ws"):
            nb = int(N.lib.tlsgpu_seal_workspace_bytes(self.n_records))
            self.d_ws = [DeviceBuffer(nb) for _ in self.launches]  # one per launch: variants may run concurrently
        for i, (var, d_ch, nch) in enumerate(self.launches):
            s = None if not streams else streams[i % len(streams)]
            ws = self.d_ws[i]
            N.call("tlsgpu_seal_dev", d_ch.ptr, nch, self.d_recs.ptr, self.n_records, self.d_pt.ptr, self.d_pt.nbytes,
                   self.d_wire.ptr, self.d_wire.nbytes, self.d_states.ptr, self.d_states.nbytes // N.CONN_STATE_BYTES,
                   self.d_len.ptr, var, ws.ptr, ws.nbytes, s.handle if s else None)

    # ------------------------------------------------------------ open direction
    def open_setup(self):
        """Open descriptors for the sealed wire arena: record r's body at
        wire_off+5, its plaintext back to pt_off of a second arena; read states
        start from the initial states (what the peer's read side holds)."""
        body = np.clip(self.wire_len - 5, 0, None)
        # the open path writes the whole decrypted body (payload | MAC | padding) after the
        # explicit IV: give each record the wire slot's room, 16-byte aligned
        self.opt_off = (self.wire_off - 11).astype(np.uint64)
        assert int((self.opt_off + body).max(initial=0)) <= self.wire_bytes
        recs = make_open_records(self.wire_off + 5, self.opt_off, body, ContentType.application_data)
        self.d_orecs = DeviceBuffer(ctypes.sizeof(recs))
        self.d_orecs.upload(np.frombuffer(recs, dtype=np.uint8))
        self.d_opt = DeviceBuffer(self.wire_bytes)
        self.d_ostatus = DeviceBuffer(4 * self.n_records)
        self.d_ostates = DeviceBuffer(self.d_states0.nbytes)
        # one open workspace per launch: variants may run concurrently on separate streams
        self.d_ows = [DeviceBuffer(max(open_workspace_bytes(self.n_records), 16)) for _ in self.launches]
        return self

    def opened_plaintext_matches(self):
        """Every record's opened payload equals its plaintext (host compare)."""
        got, ref = self.d_opt.download(), self.d_pt.download()
        for r in range(self.n_records):
            n, a, b = int(self.pt_len[r]), int(self.opt_off[r]), int(self.pt_off[r])
            if not np.array_equal(got[a:a + n], ref[b:b + n]):
                return False
        return True

    def open_launch(self, stream=None, reset=True, streams=None):
        """Open every record of the wire arena once (one call per variant; with several
        streams the variants run concurrently -- they touch disjoint records and states)."""
        if reset:
            N.call("tlsgpu_memcpy_d2d", self.d_ostates.ptr, self.d_states0.ptr, self.d_ostates.nbytes,
                   stream.handle if stream else None)
        for i, (var, d_ch, nch) in enumerate(self.launches):
            s = streams[i % len(streams)] if streams else stream
            open_dev(d_ch, nch, self.d_orecs, self.n_records, self.d_wire, self.d_opt, self.d_ostates,
                     self.d_ostatus, var, self.d_ows[i], s)

    def dominant_kernel(self):
        """Name (rocprof stem) of the kernel that dominates the first launch."""
        var, _, nch = self.launches[0]
        c, m = var & 0xff, (var >> 8) & 0xff
        if c in (N.CIPHER_AES128, N.CIPHER_AES256) and m in (N.MAC_SHA1, N.MAC_SHA256):
            from .recordlayer import seal_cipher_kernel
            return seal_cipher_kernel(var, nch)  # the layout the library picks for this many chains
        if c == N.CIPHER_3DES:
            # split path: bench.py's events bracket the whole 3DES seal call (prefix + MAC +
            # tdes4_kernel), which tdes4_kernel dominates
            return "tdes4_kernel"
        return "rc4_seal_kernel"

    def aes_lookups(self):
        """LDS T-table lookups of one seal call when every launch is an AES suite:
        16 per round per 16-byte block (4 state columns x 4 tables), NR rounds,
        blocks = explicit IV + body of every sealed record = (wire_len - 5) / 16.
        None for workloads with RC4 / 3DES launches."""
        nr = {N.CIPHER_AES128: 10, N.CIPHER_AES256: 14}
        if any((var & 0xff) not in nr for var, _, _ in self.launches):
            return None
        blocks = np.maximum(self.wire_len.astype(np.int64) - 5, 0) // 16
        return int(16 * nr[self.launches[0][0] & 0xff] * int(blocks.sum())) if len(
            {var & 0xff for var, _, _ in self.launches}) == 1 else None

    def cipher_state_bytes(self):
        """Connection-state bytes the cipher phase must move per launch: per chain the round
        keys it encrypts with (AES: 16 (NR+1); 3DES: 3 x 128), the CBC residue read and
        written and the fixedIVBlock (16 + 16 + 16) -- each connection has its own keys, so
        these are algorithmic for workloads of many one-record connections (cfg3).  0 for
        RC4-only batches."""
        per = {N.CIPHER_AES128: 176 + 48, N.CIPHER_AES256: 240 + 48, N.CIPHER_3DES: 384 + 24}
        tot = 0
        for var, _, _ in self.launches:
            tot += per.get(var & 0xff, 0)
        return int(tot * self.n_chains // max(1, len(self.launches)))

    def free(self):
        for name in ("d_pt", "d_wire", "d_len", "d_recs", "d_states", "d_states0", "d_orecs", "d_opt", "d_ostatus",
                     "d_ostates"):
            b = getattr(self, name, None)
            if b is not None:
                b.free()
        for b in getattr(self, "d_ws", []) + getattr(self, "d_ows", []):
            b.free()
        for _, d, _ in getattr(self, "launches", []):
            d.free()


def _rng_bytes(rng, n, k):
    return [rng.bytes(k) for _ in range(n)]


def cfg2(n=65536, pt_len=16384, seed=2):
    rng = np.random.default_rng(seed)
    key, mk, fiv = rng.bytes(16), rng.bytes(20), rng.bytes(16)
    ivs = np.frombuffer(rng.bytes(16 * n), dtype=np.uint8).reshape(n, 16)
    g = Group("AES128-SHA", (3, 3), [key], ivs, [mk], [fiv], np.arange(n, dtype=np.uint64), 1, pt_len)
    return Workload("cfg2: %d x %d B records, TLS_RSA_WITH_AES_128_CBC_SHA, TLS 1.2, per-record IV" % (n, pt_len),
                    [g], seed)


def cfg3(n=1048576, pt_len=1434, seed=3, pt_align=16):
    rng = np.random.default_rng(seed)
    key, mk, fiv = rng.bytes(32), rng.bytes(32), rng.bytes(16)
    ivs = np.frombuffer(rng.bytes(16 * n), dtype=np.uint8).reshape(n, 16)
    g = Group("AES256-SHA256", (3, 3), [key], ivs, [mk], [fiv], np.arange(n, dtype=np.uint64), 1, pt_len)
    name = "cfg3: %d x %d B records, TLS_RSA_WITH_AES_256_CBC_SHA256, TLS 1.2" % (n, pt_len)
    if pt_align != 16:
        name += ", plaintext records %d-B aligned" % pt_align
    return Workload(name, [g], seed, pt_align=pt_align)


def cfg4(nconn=4096, recs_per_conn=256, pt_len=16384, seed=4, rank=0, world=1):
    """Connection-sharded: this rank owns connections [rank::world]."""
    rng = np.random.default_rng(seed)
    keys = _rng_bytes(rng, nconn, 16)
    mks = _rng_bytes(rng, nconn, 20)
    fivs = _rng_bytes(rng, nconn, 16)
    ivs = np.frombuffer(rng.bytes(16 * nconn), dtype=np.uint8).reshape(nconn, 16)
    mine = np.arange(rank, nconn, world)
    g = Group("AES128-SHA", (3, 3), [keys[i] for i in mine], ivs[mine], [mks[i] for i in mine],
              [fivs[i] for i in mine], np.zeros(len(mine), dtype=np.uint64), recs_per_conn, pt_len)
    per_conn = recs_per_conn * _round_up(pt_len, 16)
    return Workload("cfg4: %d conns x %d records of %d B, AES128-SHA, chained (rank %d/%d)"
                    % (nconn, recs_per_conn, pt_len, rank, world), [g], seed,
                    chain_stream_start=mine.astype(np.uint64) * per_conn)


def cfg5(n=65536, pt_len=16384, seed=5):
    rng = np.random.default_rng(seed)
    half = n // 2
    k_rc4, mk1 = rng.bytes(16), rng.bytes(20)
    k_des, mk2, fiv = rng.bytes(24), rng.bytes(20), rng.bytes(8)
    ivs = np.frombuffer(rng.bytes(8 * (n - half)), dtype=np.uint8).reshape(n - half, 8)
    g1 = Group("RC4-SHA", (3, 3), [k_rc4], None, [mk1], None, np.arange(half, dtype=np.uint64), 1, pt_len)
    g2 = Group("3DES-SHA", (3, 3), [k_des], ivs, [mk2], [fiv], np.arange(half, n, dtype=np.uint64), 1, pt_len)
    order = rng.permutation(n)  # interleave the two suites in the arenas
    return Workload("cfg5: %d x %d B records, RC4-SHA / 3DES-EDE-CBC-SHA interleaved" % (n, pt_len), [g1, g2], seed,
                    rec_order=order)


CONFIGS = {"cfg2": cfg2, "cfg3": cfg3, "cfg4": cfg4, "cfg5": cfg5}
