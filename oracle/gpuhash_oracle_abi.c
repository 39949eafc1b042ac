/*
 * oracle/gpuhash_oracle_abi.c -- the include/gpuhash.h entry points the miner program
 * uses, implemented on the CPU oracle (oracle/hash_oracle.c).
 *
 * TEST INFRASTRUCTURE ONLY.  tests/test_native_miner.py links the miner program
 * (bitcoin-miner_amd/csrc/miner_main.cpp) against this file, in a temporary
 * directory, to test the program's LSP / JSON / failure handling on machines without a
 * GPU.  The product miner (bitcoin-miner_amd/lib/gpuhash_miner) links the real
 * libgpuhash.so; nothing under bitcoin-miner_amd/ builds or loads this file.
 *
 * Test hooks: a message equal to "__gpuhash_test_ehip__" makes gpuhash_min return
 * GPUHASH_EHIP (a device error), "__gpuhash_test_einval__" GPUHASH_EINVAL (an argument
 * error), so the miner's exit-and-requeue paths can be driven over LSP.
 */
#include <stdlib.h>
#include <string.h>

#include "gpuhash.h"

int oracle_min(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, uint64_t *out_hash,
               uint64_t *out_nonce);
uint64_t oracle_hash(const uint8_t *msg, size_t len, uint64_t nonce);

struct gpuhash_ctx {
    int unused;
};

int gpuhash_open(const int *devices, int ndevices, gpuhash_ctx **out) {
    (void)devices;
    if (!out || ndevices < 0) return GPUHASH_EINVAL;
    *out = (gpuhash_ctx *)calloc(1, sizeof(gpuhash_ctx));
    return *out ? GPUHASH_OK : GPUHASH_ENOMEM;
}

int gpuhash_min(gpuhash_ctx *ctx, const uint8_t *msg, size_t msg_len, uint64_t lower, uint64_t upper,
                uint64_t *out_hash, uint64_t *out_nonce) {
    static const char ehip[] = "__gpuhash_test_ehip__", einval[] = "__gpuhash_test_einval__";
    if (!ctx || !out_hash || !out_nonce || (msg_len && !msg) || lower > upper) return GPUHASH_EINVAL;
    if (msg_len > GPUHASH_MAX_MSG) return GPUHASH_ETOOLONG;
    if (msg_len == sizeof ehip - 1 && memcmp(msg, ehip, msg_len) == 0) return GPUHASH_EHIP;
    if (msg_len == sizeof einval - 1 && memcmp(msg, einval, msg_len) == 0) return GPUHASH_EINVAL;
    return oracle_min(msg, msg_len, lower, upper, out_hash, out_nonce) ? GPUHASH_EINVAL : GPUHASH_OK;
}

uint64_t gpuhash_hash_cpu(const uint8_t *msg, size_t msg_len, uint64_t nonce) {
    return oracle_hash(msg, msg_len, nonce);
}

void gpuhash_close(gpuhash_ctx *ctx) { free(ctx); }

const char *gpuhash_strerror(int rc) {
    switch (rc) {
        case GPUHASH_OK: return "ok";
        case GPUHASH_EINVAL: return "invalid argument";
        case GPUHASH_ENODEV: return "no device";
        case GPUHASH_EHIP: return "HIP runtime error (oracle test hook)";
        case GPUHASH_ETOOLONG: return "message longer than GPUHASH_MAX_MSG";
        case GPUHASH_ENOMEM: return "out of memory";
        default: return "unknown gpuhash error";
    }
}
