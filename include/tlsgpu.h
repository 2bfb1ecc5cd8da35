/*
 * tlsgpu.h -- C ABI of libtlsgpu.so, the MI355X (gfx950) TLS record-layer
 * bulk-crypto engine.  Plain pointers and sizes only; no torch/HIP types leak
 * through (streams and events are opaque handles).
 *
 * What each entry point replaces in the reference (trevp/tlslite 0.4.9, paths
 * relative to the repository root):
 *
 *   tlsgpu_conn_state_init ... tlsrecordlayer.py:1127-1149 (_calcPendingStates:
 *                              createHMAC / createAES / createRC4 /
 *                              createTripleDES + fixedIVBlock) and
 *                              mathtls.py:116-151 (createHMAC, MAC_SSL)
 *   tlsgpu_seal_dev .......... tlsrecordlayer.py:538-617 (_sendMsg seal block:
 *                              MAC :567-586, explicit IV :594-595, padding
 *                              :597-606, encrypt :608/:613, header :616-617),
 *                              batched over many records / connections
 *   tlsgpu_host_pipeline_seal  the same from host socket buffers: the whole
 *                              write path of :538-620 (seal + the socket-buffer
 *                              hand-off) with the PCIe copies overlapped
 *   tlsgpu_open_dev .......... tlsrecordlayer.py:958-1044 (_decryptRecord)
 *   tlsgpu_frame_dev ......... tlsrecordlayer.py:832-876 (_getNextRecord's header
 *                              parse; RecordHeader3.parse, messages.py:44-49),
 *                              batched over connections' received bytes
 *   tlsgpu_host_pipeline_open  the receive path from host socket buffers: the
 *                              recv loops :832-893, framing and _decryptRecord
 *                              :958-1044, with the PCIe copies overlapped
 *   tlsgpu_cipher_dev ........ utils/python_aes.py:20-69, utils/python_rc4.py:25-41,
 *                              utils/openssl_tripledes.py:29-47 (the stateful
 *                              cipher-object encrypt/decrypt behind
 *                              utils/cipherfactory.py:31-102)
 *   tlsgpu_derive_states_dev . tlsrecordlayer.py:1061-1149 (_calcPendingStates:
 *                              key block PRF :1097-1114, slicing :1117-1126,
 *                              cipher/MAC objects :1127-1136, side :1138-1143)
 *                              and mathtls.py:24-82 (P_hash, PRF, PRF_1_2,
 *                              PRF_SSL, calcMasterSecret), batched over
 *                              connections on the device
 *   tlsgpu_conn_state_get_* .. the state tlslite keeps in python objects:
 *                              Python_AES.IV (python_aes.py:44), Python_RC4.S/i/j
 *                              (python_rc4.py:21-23,36-37), _ConnectionState.seqnum
 *                              (tlsrecordlayer.py:31-37)
 *
 * Conventions: every function returns 0 on success or a negative error code
 * (TLSGPU_E*).  "_dev" functions take DEVICE pointers and are asynchronous on
 * the given stream (NULL = the default stream of the current device).
 *
 * Bounds (ABI 6): the batch seal / open calls take the byte size of each arena and
 * the number of connection states.  The descriptors live in device memory, so they
 * are checked on the device, per record: a record whose plaintext or wire range leaves
 * its arena, or any record of a chain whose state index is >= nstates, gets
 * TLSGPU_EINVAL in wire_len / status -- nothing of it is read or written, its state is
 * not touched and no seqnum is consumed (the reference refuses bad lengths at the object
 * boundary: utils/aes.py:28-34, codec.py:19-20).  Records of a chain past nrecords are
 * ignored.
 */
#ifndef TLSGPU_H
#define TLSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TLSGPU_ABI_VERSION 7

/* ---- suite components (tlsrecordlayer.py:1063-1095, constants.py:159-201) */
enum {
    TLSGPU_CIPHER_AES128 = 1, /* aes128Suites: key 16, IV 16 */
    TLSGPU_CIPHER_AES256 = 2, /* aes256Suites: key 32, IV 16 */
    TLSGPU_CIPHER_RC4 = 3,    /* rc4Suites:    key 16, no IV */
    TLSGPU_CIPHER_3DES = 4,   /* tripleDESSuites: key 24, IV 8 */
    TLSGPU_CIPHER_AES192 = 5  /* no suite uses it; raw cipher objects only (aes.py:8 allows 24-byte keys) */
};
enum {
    TLSGPU_MAC_SHA1 = 1,   /* shaSuites, 20-byte MAC */
    TLSGPU_MAC_SHA256 = 2, /* sha256Suites, 32-byte MAC (TLS 1.2 only) */
    TLSGPU_MAC_MD5 = 3     /* md5Suites, 16-byte MAC */
};
/* per-record fault flags (constants.py:310-359; tlsrecordlayer.py:585-586,603-604) */
enum { TLSGPU_FAULT_BAD_MAC = 1, TLSGPU_FAULT_BAD_PADDING = 2 };

/* error / status codes */
enum {
    TLSGPU_OK = 0,
    TLSGPU_EINVAL = -1,     /* bad argument (key/IV length, size, variant) */
    TLSGPU_EHIP = -2,       /* HIP runtime error; see tlsgpu_last_error() */
    TLSGPU_ENODEV = -3,     /* no GPU / bad device ordinal */
    TLSGPU_ETOOBIG = -4,    /* record body would not fit the 16-bit length (codec.py:19-20) */
    TLSGPU_EMISMATCH = -5,  /* connection state does not match the launch variant */
    TLSGPU_EFRAME = -6,     /* received bytes are not a TLS record header: the first byte is no
                             * content type (tlsrecordlayer.py:850-857 raises SyntaxError) */
    TLSGPU_EABRUPT = -7,    /* receive framing (ABI 7): a record header announcing an empty body --
                             * the reference's body loop calls sock.recv(0), gets b"" and raises
                             * TLSAbruptCloseError (tlsrecordlayer.py:877-889): the connection ends
                             * there, the empty record is not framed */
    /* open-path per-record status (alerts, tlsrecordlayer.py:964-1042) */
    TLSGPU_ALERT_BAD_RECORD_MAC = -20,
    TLSGPU_ALERT_DECRYPTION_FAILED = -21,
    /* open with TLSGPU_CHAIN_STOP_ON_ALERT: not opened, an earlier record of the
     * chain raised an alert (the reference sends the alert and closes the
     * connection there: tlsrecordlayer.py:1039-1042 -> _sendError) */
    TLSGPU_ALERT_SKIPPED = -22,
    /* receive framing: a header announced more than 18432 body bytes (record_overflow,
     * tlsrecordlayer.py:871-873) */
    TLSGPU_ALERT_RECORD_OVERFLOW = -23
};

/* Launch variant = one (cipher, MAC, SSL3-or-TLS) kernel instantiation.
 * Records of different variants go in different launches (or streams). */
#define TLSGPU_VARIANT(cipher, mac, ssl3) ((uint32_t)(cipher) | ((uint32_t)(mac) << 8) | ((uint32_t)((ssl3) ? 1 : 0) << 16))

/* ---- per-connection state: device-resident, updated in place by the
 * kernels so that consecutive batches equal one long tlslite connection.
 * Fields are private to the library except through the accessors below. */
#define TLSGPU_CONN_STATE_BYTES 2048
typedef struct tlsgpu_conn_state {
    uint8_t opaque[TLSGPU_CONN_STATE_BYTES];
} __attribute__((aligned(16))) tlsgpu_conn_state;

/* One record to seal.  Plaintext at pt + pt_off (pt_len bytes); the wire
 * record (5-byte header + body) is written at wire + wire_off.  Fast path:
 * pt_off % 16 == 0 and (wire_off + 5) % 16 == 0; any other alignment is
 * correct but slower.  pt_len == 0 writes nothing and consumes no seqnum
 * (tlsrecordlayer.py:551-556). */
typedef struct tlsgpu_record {
    uint64_t pt_off;
    uint64_t wire_off;
    uint32_t pt_len;
    uint8_t content_type; /* 23 application_data, 21 alert, 22 handshake ... */
    uint8_t flags;        /* TLSGPU_FAULT_* */
    uint16_t reserved;
} tlsgpu_record;

/* A run of records of ONE connection, sealed (or opened) in order (CBC
 * residue, RC4 keystream and seqnum carried from record to record).
 * Independent chains run in parallel; a record must belong to exactly one
 * chain. */
#define TLSGPU_CHAIN_STOP_ON_ALERT 1u /* open: records after the first alert are not
                                         opened (status TLSGPU_ALERT_SKIPPED), the state
                                         stays as the failing record left it and is marked
                                         closed: every later open of that state reports
                                         TLSGPU_ALERT_SKIPPED (round 5; state init clears
                                         the mark) */
typedef struct tlsgpu_chain {
    uint32_t state;    /* index into the states array */
    uint32_t first;    /* first record index */
    uint32_t count;    /* number of records */
    uint32_t flags;    /* TLSGPU_CHAIN_* (0: every record opened, as successive
                          _decryptRecord calls; seal ignores it) */
} tlsgpu_chain;

/* One record to open.  Body (ciphertext, header already parsed) at
 * wire + ct_off, ct_len bytes; the plaintext is written at pt + pt_off. */
typedef struct tlsgpu_open_record {
    uint64_t ct_off;
    uint64_t pt_off;
    uint32_t ct_len;
    uint8_t content_type;
    uint8_t reserved[3];
} tlsgpu_open_record;

/* Raw cipher-object span (factory surface): encrypt/decrypt len bytes of
 * in + off into out + off with connection state `state`. */
typedef struct tlsgpu_span {
    uint64_t off;
    uint32_t len;
    uint32_t state;
} tlsgpu_span;

/* One connection's post-handshake key material: the inputs of
 * _calcPendingStates (tlsrecordlayer.py:1061) and, with
 * TLSGPU_DERIVE_PREMASTER, of calcMasterSecret (mathtls.py:70). */
#define TLSGPU_DERIVE_PREMASTER 1 /* secret is the 48-byte premaster secret */
#define TLSGPU_KEY_BLOCK_MAX 160  /* 2 * (32 + 32 + 16): AES256-SHA256 */
typedef struct tlsgpu_derive_desc {
    uint8_t secret[48];        /* master secret (or premaster, see flags) */
    uint8_t client_random[32];
    uint8_t server_random[32];
    uint8_t fixed_iv[16];      /* this side's fixedIVBlock (first IV-length bytes; TLS >= 1.1 block ciphers) */
    uint16_t suite;            /* CipherSuite id (constants.py:159-201) */
    uint8_t ver_major, ver_minor;
    uint8_t client;            /* 1: this side is the client (self._client, tlsrecordlayer.py:1138) */
    uint8_t flags;             /* TLSGPU_DERIVE_* */
    uint8_t reserved[2];
} tlsgpu_derive_desc;

typedef struct tlsgpu_stream_s *tlsgpu_stream;
typedef struct tlsgpu_event_s *tlsgpu_event;

/* ---- library / device ---------------------------------------------------- */
int tlsgpu_abi_version(void);
const char *tlsgpu_last_error(void);
int tlsgpu_device_count(int *n);
int tlsgpu_set_device(int ordinal);
int tlsgpu_get_device(int *ordinal);
int tlsgpu_device_synchronize(void);
/* fills *name (cap bytes) with the device arch name, e.g. "gfx950" */
int tlsgpu_device_arch(int ordinal, char *name, size_t cap);
/* compute units of device `ordinal` (the seal kernels size their layouts per CU) */
int tlsgpu_device_cu_count(int ordinal, int *n);

/* ---- memory ------------------------------------------------------------- */
int tlsgpu_malloc(void **dptr, size_t bytes);
int tlsgpu_free(void *dptr);
int tlsgpu_host_alloc(void **hptr, size_t bytes); /* pinned host memory */
int tlsgpu_host_free(void *hptr);
int tlsgpu_memcpy_h2d(void *dst, const void *src, size_t bytes, tlsgpu_stream s);
int tlsgpu_memcpy_d2h(void *dst, const void *src, size_t bytes, tlsgpu_stream s);
int tlsgpu_memcpy_d2d(void *dst, const void *src, size_t bytes, tlsgpu_stream s);
int tlsgpu_memset(void *dptr, int value, size_t bytes, tlsgpu_stream s);

/* ---- streams / events ---------------------------------------------------- */
int tlsgpu_stream_create(tlsgpu_stream *s);
/* ABI 5: a stream at high (high != 0) or normal priority.  The HIP runtime maps a process's
 * streams onto a few hardware queues per priority level, and kernels of one queue run in
 * submission order: two streams whose work should overlap are only certain to get separate
 * queues at different priorities (the seal pipeline's MAC / cipher streams are; DESIGN.md
 * section 6).  Replaces nothing in the reference (tlslite has no device streams). */
int tlsgpu_stream_create_priority(tlsgpu_stream *s, int high);
/* (high == 0 gives the runtime's LEAST priority level -- hipDeviceGetStreamPriorityRange's
 * "least", below the normal level of tlsgpu_stream_create streams -- so a high / low pair
 * never shares a hardware queue with each other.) */
/* waits for the stream, frees the library-owned seal / open workspaces of this stream
 * (tlsgpu_seal_dev / tlsgpu_open_dev with a NULL workspace), then destroys it */
int tlsgpu_stream_destroy(tlsgpu_stream s);
int tlsgpu_stream_synchronize(tlsgpu_stream s);
int tlsgpu_event_create(tlsgpu_event *e);
int tlsgpu_event_destroy(tlsgpu_event e);
int tlsgpu_event_record(tlsgpu_event e, tlsgpu_stream s);
int tlsgpu_event_synchronize(tlsgpu_event e);
int tlsgpu_event_elapsed_ms(float *ms, tlsgpu_event start, tlsgpu_event stop);

/* ---- connection state (host-side construction, no GPU needed) ------------
 * Equivalent of _calcPendingStates' per-direction state: key schedule of the
 * bulk cipher, HMAC ipad/opad midstates (or SSL3 MAC_SSL prefix state), CBC
 * IV, TLS>=1.1 fixedIVBlock, RC4 KSA, seqnum.  Validation mirrors the
 * reference: AES key 16/32 + IV 16 (aes.py:7-13), 3DES key 24 + IV 8
 * (tripledes.py:8-13), RC4 key 16..256 + empty IV (rc4.py:9-10,
 * cipherfactory.py:70-71); SHA256 only at TLS 1.2 (constants.py:204-210). */
int tlsgpu_conn_state_init(tlsgpu_conn_state *st, int cipher, int mac, int ver_major, int ver_minor,
                           const uint8_t *key, size_t key_len, const uint8_t *iv, size_t iv_len,
                           const uint8_t *mac_key, size_t mac_key_len, const uint8_t *fixed_iv,
                           size_t fixed_iv_len, uint64_t seqnum);
/* raw cipher context (cipher-object surface: no MAC, version 0.0) */
int tlsgpu_cipher_state_init(tlsgpu_conn_state *st, int cipher, const uint8_t *key, size_t key_len,
                             const uint8_t *iv, size_t iv_len);
int tlsgpu_conn_state_set_seqnum(tlsgpu_conn_state *st, uint64_t seqnum);
int tlsgpu_conn_state_set_iv(tlsgpu_conn_state *st, const uint8_t *iv, size_t iv_len);
int tlsgpu_conn_state_get_seqnum(const tlsgpu_conn_state *st, uint64_t *seqnum);
int tlsgpu_conn_state_get_iv(const tlsgpu_conn_state *st, uint8_t *iv, size_t cap, size_t *iv_len);
int tlsgpu_conn_state_get_rc4(const tlsgpu_conn_state *st, uint8_t S[256], uint32_t *i, uint32_t *j);
int tlsgpu_conn_state_variant(const tlsgpu_conn_state *st, uint32_t *variant);
/* wire length of a sealed record of pt_len bytes for this state (0 if pt_len==0) */
int tlsgpu_seal_wire_len(const tlsgpu_conn_state *st, uint32_t pt_len, uint32_t *wire_len);

/* ---- batch seal / open (device pointers, async on stream) ---------------
 * wire_len[r] receives the bytes written for record r (header included), 0
 * for an empty record, or a negative TLSGPU_E* code.  All chains of one
 * launch must use connection states of `variant`; `records` has `nrecords`
 * entries (chains index into it). */
/* Device workspace for a seal of `nrecords` descriptors (AES / 3DES suites:
 * per record 32 B of metadata + a 64 B CBC-tail slot).  Pass it to
 * tlsgpu_seal_dev, or pass NULL there to use a library-owned workspace, one
 * per (device, stream): calls on different streams never share one. */
size_t tlsgpu_seal_workspace_bytes(uint32_t nrecords);
/* Free every library-owned seal / open workspace (the NULL-workspace buffers, one per
 * (device, stream) in use; the device is the stream's).  Waits for each device they live
 * on first; every entry is dropped even when a HIP call fails (the first error is
 * returned).  tlsgpu_stream_destroy already frees its stream's buffers.  Must not run
 * concurrently with a seal / open call that passes a NULL workspace. */
int tlsgpu_release_workspaces(void);
/* number of library-owned workspaces currently allocated (diagnostics / tests) */
size_t tlsgpu_owned_workspace_count(void);
/* ABI 6: number of library-owned streams (the split open's second streams, one per device and
 * priority in use, with their events); tlsgpu_release_workspaces destroys them too */
size_t tlsgpu_owned_stream_count(void);
/* Name of the cipher-phase kernel a seal call of `nchains` chains of `variant` runs on the
 * current device (its rocprofv3 name stem, e.g. "cbc_kernel<10, false>"): the layout is
 * chosen from the chains per CU.  Diagnostics / profiling only. */
int tlsgpu_seal_cipher_kernel(uint32_t variant, uint32_t nchains, char *name, size_t cap);
/* pt: plaintext arena of pt_bytes, wire: wire arena of wire_bytes, states: nstates states
 * (ABI 6 bounds, see the top of this file) */
int tlsgpu_seal_dev(const tlsgpu_chain *chains, uint32_t nchains, const tlsgpu_record *records,
                    uint32_t nrecords, const uint8_t *pt, size_t pt_bytes, uint8_t *wire, size_t wire_bytes,
                    tlsgpu_conn_state *states, uint32_t nstates, int32_t *wire_len, uint32_t variant,
                    void *workspace, size_t workspace_bytes, tlsgpu_stream s);
/* ---- seal pipeline: successive tlsgpu_pipeline_seal calls overlap the MAC
 * phase of call k+1 with the cipher phase of call k (AES suites; two
 * library-owned streams, three workspaces in rotation, so the MAC phase may run
 * up to two calls ahead).  Inputs must be ready
 * when a call is made and stay valid, and outputs are complete, only after
 * tlsgpu_pipeline_synchronize.  Optional events bracket the cipher kernel. */
typedef struct tlsgpu_pipeline_s *tlsgpu_pipeline;
int tlsgpu_pipeline_create(tlsgpu_pipeline *p, uint32_t max_records);
int tlsgpu_pipeline_destroy(tlsgpu_pipeline p);
int tlsgpu_pipeline_synchronize(tlsgpu_pipeline p);
int tlsgpu_pipeline_seal(tlsgpu_pipeline p, const tlsgpu_chain *chains, uint32_t nchains,
                         const tlsgpu_record *records, uint32_t nrecords, const uint8_t *pt, size_t pt_bytes,
                         uint8_t *wire, size_t wire_bytes, tlsgpu_conn_state *states, uint32_t nstates,
                         int32_t *wire_len, uint32_t variant, tlsgpu_event cipher_start, tlsgpu_event cipher_stop);

/* ---- host-buffer seal pipeline: records start and end in host socket buffers
 * (tlsrecordlayer.py:616-620 writes each sealed record to the socket).  One call
 * seals a batch whose plaintext arena, descriptors and wire arena are in HOST
 * memory; connection states stay device-resident.  The batch is cut into
 * sub-batches of consecutive chains (about chunk_bytes of plaintext each).  Four
 * library-owned streams chained per sub-batch by events: H2D copies of the sub-batches'
 * plaintext, their MAC phases, their cipher phases, D2H copies of their wire ranges --
 * so copies in both directions, the MAC phase of one sub-batch and the cipher phase of
 * the one before run at once; `depth` sub-batches are in flight.  pt_host / wire_host that
 * are pinned (tlsgpu_host_alloc) are copied directly; pageable buffers are staged
 * through library-owned pinned buffers (depth of them per direction, filled and
 * drained by the calling thread).  Sub-batch copy ranges are cut at the first
 * record offsets of the next sub-batch, so records should be laid out in chain
 * order (as tlsgpu_seal_dev callers normally do); any other layout is sealed as
 * one sub-batch.  Synchronous: wire_host and wire_len_host are complete on return.
 * Every record's wire slot must hold its sealed size (header, [explicit IV], P, MAC,
 * padding): an RC4 record that would not fit fails the call with TLSGPU_EINVAL; a CBC
 * record (whose size depends on the state's version) gets wire_len = TLSGPU_EINVAL and is
 * not sealed (no seqnum consumed).  Bytes of wire_host between records are written as
 * zeros.  A chain whose state index is >= nstates fails the call with TLSGPU_EINVAL (the
 * chains are host memory here, checked before anything is enqueued).
 * wire_len_host: nrecords int32 (as tlsgpu_seal_dev's wire_len). */
typedef struct tlsgpu_host_pipeline_s *tlsgpu_host_pipeline;
int tlsgpu_host_pipeline_create(tlsgpu_host_pipeline *p, size_t chunk_bytes, int depth);
int tlsgpu_host_pipeline_destroy(tlsgpu_host_pipeline p);
int tlsgpu_host_pipeline_seal(tlsgpu_host_pipeline p, const tlsgpu_chain *chains, uint32_t nchains,
                              const tlsgpu_record *records, uint32_t nrecords, const uint8_t *pt_host,
                              size_t pt_bytes, uint8_t *wire_host, size_t wire_bytes, tlsgpu_conn_state *states,
                              uint32_t nstates, int32_t *wire_len_host, uint32_t variant);
/* The host pipelines' large D2H copies (wire ranges, opened plaintext) go by the copy engine or
 * by the GPU's own stores into the pinned destination (tlsgpu_host_store's kernel): each pipeline
 * times them on its first call (32 MiB, ~4 ms) and keeps the stores only when the engine's D2H
 * runs below 0.7x its H2D rate and the stores are >= 1.5x faster -- in some processes the
 * engine's D2H runs at about half its usual rate while the stores do not.  TLSGPU_HOST_D2H=engine|kernel in the environment
 * forces a path.  *path: -1 not chosen yet, 0 copy engine, 1 device stores. */
int tlsgpu_host_pipeline_d2h_path(tlsgpu_host_pipeline p, int *path);
/* D2H copy by device stores, async on s: dst_host is pinned host memory (tlsgpu_host_alloc) at
 * the same address mod 16 as src_dev; TLSGPU_EINVAL otherwise. */
int tlsgpu_host_store(void *dst_host, const void *src_dev, size_t bytes, tlsgpu_stream s);

/* Batch open: status[r] = plaintext length, or TLSGPU_ALERT_* (records 0..nrecords-1;
 * a chain's records open in order on its state, as successive _decryptRecord calls).
 * A connection must not accept records after an alert: set TLSGPU_CHAIN_STOP_ON_ALERT
 * on its chain (or stop at the first negative status yourself).
 * The whole decrypted body after the explicit IV (payload | MAC | padding, ct_len - IV
 * bytes) is written at pt + pt_off: size the plaintext slots for it.
 * CBC suites (AES, 3DES) decrypt every block of every record in parallel and need a
 * workspace of tlsgpu_open_workspace_bytes(nrecords) bytes (NULL = library-owned).
 * wire: ciphertext arena of wire_bytes, pt: plaintext arena of pt_bytes, states: nstates
 * states (ABI 6 bounds: a refused record gets status TLSGPU_EINVAL and is treated as if it
 * were not in the batch).
 * Large batches open in parts on a library-owned second stream beside the caller's
 * (DESIGN.md section 3.4).  Limits of that stream: one per (device, priority), so
 * split opens issued at once on different caller streams of one priority run their decrypt
 * passes one after another; and a caller stream under HIP graph capture pulls it into the
 * capture.  tlsgpu_release_workspaces destroys it. */
size_t tlsgpu_open_workspace_bytes(uint32_t nrecords);
int tlsgpu_open_dev(const tlsgpu_chain *chains, uint32_t nchains, const tlsgpu_open_record *records,
                    uint32_t nrecords, const uint8_t *wire, size_t wire_bytes, uint8_t *pt, size_t pt_bytes,
                    tlsgpu_conn_state *states, uint32_t nstates, int32_t *status, uint32_t variant,
                    void *workspace, size_t workspace_bytes, tlsgpu_stream s);
/* ABI 6: how CBC-suite opens are split (process-wide).
 * mode TLSGPU_OPEN_SPLIT_AUTO (the default): chain-range parts for large batches of short
 * chains, one pass otherwise; CHAINS: chain-range parts for every batch of at least
 * min_records records (tests); NONE: every pass once on the caller's stream; BLOCKS (3DES
 * suites; AES opens take NONE): block-range parts -- every record's tail and the padding
 * pass first, then block ranges of every record beside the MAC of the payload decrypted so
 * far -- for every batch of at least min_records records.  AUTO picks BLOCKS for 3DES
 * batches of >= 128 records per CU that it does not split by chain. */
enum { TLSGPU_OPEN_SPLIT_AUTO = 0, TLSGPU_OPEN_SPLIT_CHAINS = 1, TLSGPU_OPEN_SPLIT_NONE = 2,
       TLSGPU_OPEN_SPLIT_BLOCKS = 3 };
int tlsgpu_set_open_parts(int mode, int64_t min_records);
/* Receive path from HOST socket buffers (ABI 7): connection i's received bytes are
 * rx_host[conns[i].off, + conns[i].len) -- what the reference's sock.recv loops gather
 * (tlsrecordlayer.py:832-893) -- and they are framed (as tlsgpu_frame_dev) and opened (as
 * tlsgpu_open_dev, :958-1044) on the device, in sub-batches of consecutive connections of
 * about chunk_bytes received bytes: H2D copy, framing, open and D2H copy of `depth`
 * sub-batches overlap on the pipeline's streams.  Results, as one tlsgpu_frame_dev +
 * tlsgpu_open_dev over every connection would give them:
 *   records_host[0 .. *total_host)  the framed records in connection order (ct_off = pt_off =
 *                                   the body's offset in rx_host), at most max_records;
 *   status_host[r]                  record r's open status (plaintext length or TLSGPU_ALERT_*);
 *   pt_host + pt_off                record r's decrypted body after the explicit IV (payload |
 *                                   MAC | padding, as tlsgpu_open_dev writes it); pt_bytes >=
 *                                   rx_bytes.  pt_host bytes of each sub-batch's received range
 *                                   [first span, last span end) that hold no opened body come
 *                                   back zero;
 *   chains_host[i], consumed_host[i], frame_status_host[i]  as tlsgpu_frame_dev's chains /
 *                                   consumed / status (chains_host[i].first indexes records_host).
 * states: DEVICE array of nstates read states (updated in place); every connection of the call
 * must use its own state, of `variant`.  Host arrays may be pinned (copied directly) or
 * pageable (staged through the pipeline's pinned buffers).  Synchronous. */
int tlsgpu_host_pipeline_open(tlsgpu_host_pipeline p, const uint8_t *rx_host, size_t rx_bytes,
                              const tlsgpu_span *conns, uint32_t n, uint32_t chain_flags, uint8_t *pt_host,
                              size_t pt_bytes, tlsgpu_conn_state *states, uint32_t nstates, uint32_t variant,
                              tlsgpu_open_record *records_host, uint32_t max_records, tlsgpu_chain *chains_host,
                              uint32_t *consumed_host, int32_t *frame_status_host, int32_t *status_host,
                              uint32_t *total_host);
/* ---- receive framing on the device (ABI 6, round 5; ABI 7: TLSGPU_EABRUPT, 64-bit
 * workspace sums): _getNextRecord's header parse
 * (tlsrecordlayer.py:832-876; RecordHeader3.parse, messages.py:44-49) for n connections'
 * received bytes in one arena of stream_bytes, connection i's at [conns[i].off, conns[i].off +
 * conns[i].len).  Each complete record becomes one tlsgpu_open_record {ct_off = pt_off = its
 * body's offset in the arena, ct_len, content_type}, in connection order from records[0];
 * chains[i] = {conns[i].state, first, count, chain_flags}; consumed[i] = the bytes of the
 * connection's framed records (an incomplete trailing record stays for the next call);
 * status[i] = the number of records framed, or TLSGPU_ALERT_RECORD_OVERFLOW (a header
 * announcing more than 18432 body bytes: the records before it are framed, the connection
 * stops there), TLSGPU_EFRAME (a record starting with a byte that is no content type 20-23;
 * SSLv2 headers belong to the handshake, which is out of scope), TLSGPU_EABRUPT (a header
 * announcing an empty body: the reference raises TLSAbruptCloseError there, so the records
 * before it are framed and the connection stops), TLSGPU_EINVAL (the span
 * leaves the arena).  Records past max_records are not framed (consumed[] stops before
 * them).  total (device, one uint32) = records framed (0 for n = 0).  The result feeds tlsgpu_open_dev
 * directly (nrecords = max_records, or *total read back), with a plaintext arena of
 * stream_bytes.  Everything is device memory; workspace: tlsgpu_frame_workspace_bytes(n),
 * 8-byte aligned. */
size_t tlsgpu_frame_workspace_bytes(uint32_t n);
int tlsgpu_frame_dev(const uint8_t *stream, size_t stream_bytes, const tlsgpu_span *conns, uint32_t n,
                     tlsgpu_open_record *records, uint32_t max_records, tlsgpu_chain *chains,
                     uint32_t chain_flags, uint32_t *consumed, int32_t *status, uint32_t *total,
                     void *workspace, size_t workspace_bytes, tlsgpu_stream s);
/* raw stateful encrypt (decrypt=0) / decrypt (decrypt=1) of spans; one span
 * per state per launch (a state's spans in one launch run in array order). */
int tlsgpu_cipher_dev(const tlsgpu_span *spans, uint32_t nspans, const uint8_t *in, uint8_t *out,
                      tlsgpu_conn_state *states, int cipher, int decrypt, tlsgpu_stream s);

/* ---- synthetic input (bench / tests): byte i = byte (i&7) of
 * splitmix64(seed + (i>>3)), little-endian, for i in [start, start+bytes). */
/* Batched key derivation: for each descriptor, derive the key block and
 * build this side's pending write and read states (device pointers,
 * n states each), exactly as tlsgpu_conn_state_init would from the same
 * slices (the read state gets an all-zero fixed IV, which only the sender
 * uses).  master_out (48 B per connection) and key_block_out
 * (TLSGPU_KEY_BLOCK_MAX B per connection, zero-padded) may be NULL.
 * status[i] = 0, or TLSGPU_EINVAL for an unknown suite / bad version. */
int tlsgpu_derive_states_dev(const tlsgpu_derive_desc *descs, uint32_t n, tlsgpu_conn_state *write_states,
                             tlsgpu_conn_state *read_states, uint8_t *master_out, uint8_t *key_block_out,
                             int32_t *status, tlsgpu_stream s);
int tlsgpu_fill_pattern(uint8_t *dptr, size_t bytes, uint64_t seed, uint64_t start, tlsgpu_stream s);

#ifdef __cplusplus
}
#endif
#endif /* TLSGPU_H */
