// server_main.cpp -- the server program of the reference, compiled.
//
// The reference's server is a Go program whose body is a stub
// (src/github.com/cmu440/bitcoin/server/server.go:8-16, "TODO: implement this!" at :15);
// p1.pdf pp.13-15 specifies it: accept miners (Join) and clients (Request) over LSP,
// split each request into jobs, farm them to miners, fold their Results with the
// (hash, nonce) key, answer the client; reassign a lost miner's job, drop a lost
// client's work.  This is bitcoin-miner_amd/bitcoin/server.py's scheduler in C++ over
// lsp_native.h, so a whole system (this server, lib/gpuhash_miner, any client) runs as
// compiled programs; it interoperates with the Python programs message for message.
//
//   gpuhash_server port
//     GPUHASH_JOB_SIZE     nonces per job (default 2^34, ~0.5 s on one MI355X)
//     GPUHASH_MINER_DEPTH  jobs a miner may hold at once (default 1; server.py's Scheduler)
//     GPUHASH_SERVER_LOG   log joins, requests and failure handling to stderr
//     LSP_EPOCH_LIMIT / LSP_EPOCH_MILLIS / LSP_WINDOW_SIZE, LSPNET_SERVER_{READ,WRITE}_DROP
//
// Scheduling: an idle miner (fewest jobs held, then longest since its last job) gets the
// next job of the request with the fewest jobs in flight, then the least work left to hand
// out (shortest remaining first: a short request arriving while a long one holds every
// miner is not kept waiting, and equal requests finish in turn), then the oldest.  Failures: a
// lost miner's jobs go back to the front of their requests' queues, at most
// MAX_REQUEUES times per job, after which the request is abandoned and its client
// disconnected; a lost client's requests are dropped and late results ignored.  A
// Request is served only if 0 <= Lower <= Upper <= 2^64-1 and Data fits the engine;
// otherwise the client's connection is closed.  stdout is never written.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <string>
#include <vector>

#include "gpuhash.h"  // GPUHASH_MAX_MSG only: the server never loads the engine
#include "lsp_native.h"

namespace {

using lspn::BtcMsg;

constexpr int kMaxRequeues = 3;

bool g_log = false;

void logf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void logf(const char* fmt, ...) {
    if (!g_log) return;
    va_list ap;
    va_start(ap, fmt);
    std::fputs("server: ", stderr);
    std::vfprintf(stderr, fmt, ap);
    std::fputc('\n', stderr);
    va_end(ap);
}

uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* e = std::getenv(name);
    if (!e || !*e) return dflt;
    char* end = nullptr;
    unsigned long long v = std::strtoull(e, &end, 10);
    return (end && *end == '\0' && v > 0) ? (uint64_t)v : dflt;
}

struct Job {
    uint64_t req, lo, hi;
    int requeues = 0;
};

struct Request {
    uint64_t id;
    long long client;
    std::string data;
    uint64_t next_lo, upper;
    bool cut_all = false;  // every nonce is in some job (next_lo cannot pass 2^64-1)
    std::deque<Job> requeued;
    int inflight = 0;
    bool has_best = false;
    uint64_t bh = 0, bn = 0;

    bool has_pending() const { return !requeued.empty() || !cut_all; }
    // nonces not yet handed to a miner (up to 2^64: hence 128 bits)
    unsigned __int128 remaining() const {
        unsigned __int128 n = cut_all ? 0 : (unsigned __int128)upper - next_lo + 1;
        for (const Job& j : requeued) n += (unsigned __int128)j.hi - j.lo + 1;
        return n;
    }
    Job pop_job(uint64_t size) {
        if (!requeued.empty()) {
            Job j = requeued.front();
            requeued.pop_front();
            return j;
        }
        const uint64_t lo = next_lo;
        const uint64_t hi = upper - lo < size - 1 ? upper : lo + (size - 1);
        if (hi == upper) cut_all = true;
        else next_lo = hi + 1;
        return Job{id, lo, hi, 0};
    }
};

class Scheduler {
   public:
    Scheduler(uint64_t job_size, int depth) : job_size_(job_size), depth_(depth < 1 ? 1 : depth) {}

    std::deque<long long> abandoned;  // clients to disconnect

    void add_miner(long long conn) {
        if (!miners_.count(conn)) {
            miners_[conn];
            turn_[conn] = tick_++;
        }
    }

    // "" if served, else why the request was refused
    std::string add_request(long long client, const BtcMsg& m) {
        if (m.lower > m.upper)
            return "empty range: Lower " + std::to_string(m.lower) + " > Upper " + std::to_string(m.upper);
        if (m.data.size() > GPUHASH_MAX_MSG)
            return "Data is " + std::to_string(m.data.size()) + " bytes, over the engine's limit";
        // every job cut from it must fit one LSP datagram (2000-byte reads, lspnet/conn.go:35):
        // a job's bounds can have more digits than the client's Lower (but never exceed its
        // Upper), and a truncated datagram is never acked, so the job would hang
        // (bitcoin/server.py request_error)
        {
            BtcMsg job;
            job.type = lspn::Request;
            job.data = m.data;
            job.lower = job.upper = m.upper;
            const std::string frame =
                lspn::lsp_marshal(lspn::LspMsg{lspn::MsgData, 2147483647, 2147483647, true, lspn::btc_marshal(job)});
            if (frame.size() > lspn::kMaxDatagram)
                return "its jobs would not fit a " + std::to_string(lspn::kMaxDatagram) + "-byte LSP datagram";
        }
        Request r;
        r.id = next_id_++;
        r.client = client;
        r.data = m.data;
        r.next_lo = m.lower;
        r.upper = m.upper;
        requests_.emplace(r.id, std::move(r));
        return "";
    }

    // (miner, job, data) of the next dispatch; false when none
    bool next_assignment(long long& miner, Job& job, std::string& data) {
        long long best_m = 0;
        bool found = false;
        for (auto& [m, q] : miners_) {
            if ((int)q.size() >= depth_) continue;
            if (!found || q.size() < miners_[best_m].size() ||
                (q.size() == miners_[best_m].size() && turn_[m] < turn_[best_m])) {
                best_m = m;
                found = true;
            }
        }
        if (!found) return false;
        Request* r = nullptr;
        for (auto& [id, x] : requests_) {
            if (!x.has_pending()) continue;
            // fewest jobs in flight, then least work left; map order = oldest on ties
            if (!r || x.inflight < r->inflight ||
                (x.inflight == r->inflight && x.remaining() < r->remaining()))
                r = &x;
        }
        if (!r) return false;
        job = r->pop_job(job_size_);
        r->inflight++;
        miners_[best_m].push_back(job);
        turn_[best_m] = tick_++;
        miner = best_m;
        data = r->data;
        return true;
    }

    // folds a miner's Result (its oldest job); true with the client and answer when done
    bool result(long long miner, uint64_t h, uint64_t n, long long& client, uint64_t& bh, uint64_t& bn) {
        auto it = miners_.find(miner);
        if (it == miners_.end() || it->second.empty()) return false;
        Job job = it->second.front();
        it->second.pop_front();
        auto r = requests_.find(job.req);
        if (r == requests_.end()) return false;  // the client is gone: ignore the result
        Request& q = r->second;
        q.inflight--;
        if (!q.has_best || h < q.bh || (h == q.bh && n < q.bn)) {
            q.has_best = true;
            q.bh = h;
            q.bn = n;
        }
        if (q.has_pending() || q.inflight > 0) return false;
        client = q.client;
        bh = q.bh;
        bn = q.bn;
        requests_.erase(r);
        return true;
    }

    void lost(long long conn) {
        auto it = miners_.find(conn);
        if (it != miners_.end()) {
            std::deque<Job> jobs = std::move(it->second);
            miners_.erase(it);
            turn_.erase(conn);
            logf("miner %lld lost", conn);
            for (auto j = jobs.rbegin(); j != jobs.rend(); ++j) {  // oldest ends up first
                auto r = requests_.find(j->req);
                if (r == requests_.end()) continue;
                r->second.inflight--;
                if (++j->requeues > kMaxRequeues) {
                    logf("job [%llu, %llu] lost %d miners: request %llu abandoned, client %lld disconnected",
                         (unsigned long long)j->lo, (unsigned long long)j->hi, j->requeues,
                         (unsigned long long)j->req, r->second.client);
                    abandoned.push_back(r->second.client);
                    requests_.erase(r);
                    continue;
                }
                r->second.requeued.push_front(*j);
                logf("job [%llu, %llu] of request %llu requeued", (unsigned long long)j->lo,
                     (unsigned long long)j->hi, (unsigned long long)j->req);
            }
        }
        for (auto r = requests_.begin(); r != requests_.end();) {
            if (r->second.client == conn) {
                logf("client %lld lost; dropped request %llu", conn, (unsigned long long)r->first);
                r = requests_.erase(r);
            } else {
                ++r;
            }
        }
    }

   private:
    uint64_t job_size_;
    int depth_;
    uint64_t next_id_ = 1, tick_ = 0;
    std::map<uint64_t, Request> requests_;
    std::map<long long, std::deque<Job>> miners_;
    std::map<long long, uint64_t> turn_;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {  // server.go:9-13
        std::printf("Usage: ./server <port>\n");
        return 0;
    }
    g_log = std::getenv("GPUHASH_SERVER_LOG") != nullptr;
    lspn::Params params;
    lspn::Server srv(params);
    if (!srv.listen(std::atoi(argv[1]))) {
        std::fprintf(stderr, "server: cannot listen on port %s\n", argv[1]);
        return 1;
    }
    Scheduler sched(env_u64("GPUHASH_JOB_SIZE", 1ull << 34), (int)env_u64("GPUHASH_MINER_DEPTH", 1));

    auto dispatch = [&] {
        while (!sched.abandoned.empty()) {
            srv.close_conn(sched.abandoned.front());
            sched.abandoned.pop_front();
        }
        long long miner;
        Job job;
        std::string data;
        while (sched.next_assignment(miner, job, data)) {
            BtcMsg req;
            req.type = lspn::Request;
            req.data = data;
            req.lower = job.lo;
            req.upper = job.hi;
            if (!srv.write(miner, lspn::btc_marshal(req))) {
                sched.lost(miner);
                while (!sched.abandoned.empty()) {
                    srv.close_conn(sched.abandoned.front());
                    sched.abandoned.pop_front();
                }
            }
        }
    };

    for (;;) {
        lspn::Server::Event e = srv.read();
        if (e.lost) {
            logf("connection %lld %s", e.conn, e.reason == "closed" ? "closed" : ("lost (" + e.reason + ")").c_str());
            sched.lost(e.conn);
            dispatch();
            continue;
        }
        BtcMsg m;
        if (!lspn::btc_unmarshal(e.payload, m)) continue;  // not a Message: ignored
        if (m.type == lspn::Join) {
            sched.add_miner(e.conn);
            logf("conn %lld: [Join]", e.conn);
        } else if (m.type == lspn::Request) {
            std::string why = sched.add_request(e.conn, m);
            if (!why.empty()) {
                logf("conn %lld: request rejected (%s); closing the connection", e.conn, why.c_str());
                srv.close_conn(e.conn);
                continue;
            }
            logf("conn %lld: %s", e.conn, lspn::btc_describe(m).c_str());
        } else if (m.type == lspn::Result) {
            long long client;
            uint64_t h, n;
            if (sched.result(e.conn, m.hash, m.nonce, client, h, n)) {
                BtcMsg res;
                res.type = lspn::Result;
                res.hash = h;
                res.nonce = n;
                srv.write(client, lspn::btc_marshal(res));
            }
        }
        dispatch();
    }
}
