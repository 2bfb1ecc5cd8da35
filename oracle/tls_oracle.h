/* tls_oracle.h -- CPU restatement of tlslite's record seal/open (TEST
 * INFRASTRUCTURE ONLY; see tls_oracle.c header). */
#ifndef TLS_ORACLE_H
#define TLS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

enum { ORA_CIPHER_AES128 = 1, ORA_CIPHER_AES256 = 2, ORA_CIPHER_RC4 = 3, ORA_CIPHER_3DES = 4 };
enum { ORA_MAC_SHA1 = 1, ORA_MAC_SHA256 = 2, ORA_MAC_MD5 = 3 };
enum { ORA_FAULT_BAD_MAC = 1, ORA_FAULT_BAD_PADDING = 2 };
enum { ORA_ALERT_BAD_RECORD_MAC = -20, ORA_ALERT_DECRYPTION_FAILED = -21 };

typedef struct { int rounds; uint32_t ke[60]; uint32_t kd[60]; } ora_aes;

typedef struct {
    int cipher, mac, vmaj, vmin, bs;
    uint64_t seq;
    ora_aes aes;
    uint64_t des[3][16];
    uint8_t rc4_S[256];
    int rc4_i, rc4_j;
    uint8_t iv[16];
    uint8_t fixed_iv[16];
    uint8_t mac_key[64];
    int mac_key_len;
} ora_conn;

int ora_conn_init(ora_conn *c, int cipher, int mac, int vmaj, int vmin, const uint8_t *key, size_t klen,
                  const uint8_t *iv, size_t ivlen, const uint8_t *mac_key, size_t mklen,
                  const uint8_t *fixed_iv, uint64_t seq);
long ora_seal_len(const ora_conn *c, size_t n);
long ora_seal(ora_conn *c, int ctype, const uint8_t *pt, size_t n, int fault, uint8_t *out, size_t cap);
long ora_open(ora_conn *c, int ctype, uint8_t *b, size_t n, size_t *pt_off);
int ora_cipher_encrypt(ora_conn *c, uint8_t *b, size_t n);
int ora_cipher_decrypt(ora_conn *c, uint8_t *b, size_t n);
void ora_hash(int alg, const uint8_t *p, size_t n, uint8_t *out);
void ora_hmac(int alg, const uint8_t *key, size_t klen, const uint8_t *msg, size_t n, uint8_t *out);
int ora_prf(int vmin, const uint8_t *secret, size_t slen, const uint8_t *label, size_t llen,
            const uint8_t *seed, size_t seedlen, uint8_t *out, size_t length);
void ora_conn_get_iv(const ora_conn *c, uint8_t *iv16);
uint64_t ora_conn_get_seq(const ora_conn *c);
void ora_conn_get_rc4(const ora_conn *c, uint8_t *S256, int *i, int *j);
size_t ora_conn_size(void);
int ora_seal_batch(ora_conn *protos, size_t nchains, const uint32_t *chain_begin, const uint32_t *chain_count,
                   const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len, const uint8_t *ctype,
                   const uint8_t *flags,
                   uint8_t *wire, const uint64_t *wire_off, long *wire_len, int nthreads);
void ora_fill_pattern(uint8_t *p, size_t n, uint64_t seed, uint64_t start);
#endif
