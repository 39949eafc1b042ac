// Test infrastructure (tests/test_json_parity.py): reads one JSON document per line of
// stdin (hex-encoded, so any byte can travel) and prints what csrc/lsp_native.h's
// btc_unmarshal makes of it: "ERR", or "OK type lower upper hash nonce <data hex>";
// with the argument "lsp", what lsp_unmarshal makes of it: "ERR", or
// "OK type conn seq <payload hex, or - for nil>".
#include <cstdio>
#include <iostream>
#include <string>

#include "lsp_native.h"

static std::string unhex(const std::string& h) {
    std::string out;
    for (size_t i = 0; i + 1 < h.size(); i += 2) out += (char)std::stoi(h.substr(i, 2), nullptr, 16);
    return out;
}

int main(int argc, char** argv) {
    const bool lsp = argc > 1 && std::string(argv[1]) == "lsp";
    std::string line;
    while (std::getline(std::cin, line)) {
        if (lsp) {
            lspn::LspMsg m;
            if (!lspn::lsp_unmarshal(unhex(line), m)) {
                std::puts("ERR");
                continue;
            }
            std::printf("OK %lld %lld %lld ", m.type, m.conn, m.seq);
            if (!m.has_payload) std::printf("-");
            for (unsigned char c : m.payload) std::printf("%02x", c);
            std::puts("");
            continue;
        }
        lspn::BtcMsg m;
        if (!lspn::btc_unmarshal(unhex(line), m)) {
            std::puts("ERR");
            continue;
        }
        std::printf("OK %lld %llu %llu %llu %llu ", m.type, (unsigned long long)m.lower,
                    (unsigned long long)m.upper, (unsigned long long)m.hash, (unsigned long long)m.nonce);
        for (unsigned char c : m.data) std::printf("%02x", c);
        std::puts("");
    }
    return 0;
}
