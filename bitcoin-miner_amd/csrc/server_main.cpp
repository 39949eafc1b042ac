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
//     GPUHASH_JOB_SIZE     nonces per job (default: half a second of one MI355X, or one
//                          LSP epoch if shorter, a power of two: 2^34 at 2 s epochs; one
//                          epoch, 2^36, with LSP_SEND_COPIES=1; server.py default_job_size)
//     GPUHASH_MINER_DEPTH  jobs a miner may hold at once (default 3)
//     GPUHASH_COPIES       live copies of an overdue job (default 3; GPUHASH_BACKUP=0: 1)
//     GPUHASH_SERVER_LOG   log joins, requests, copies and failure handling to stderr
//     LSP_EPOCH_LIMIT / LSP_EPOCH_MILLIS / LSP_WINDOW_SIZE, LSP_SEND_COPIES (default 3),
//     LSPNET_SERVER_{READ,WRITE}_DROP
//
// Scheduling: an idle miner (fewest jobs held, then longest since its last job) gets the
// next job of the request with the fewest jobs in flight, then the least work left to hand
// out (shortest remaining first: a short request arriving while a long one holds every
// miner is not kept waiting, and equal requests finish in turn), then the oldest.  With
// nothing left to hand out, a miner holding nothing gets a copy of a job every holder of
// which is overdue by its learned rate.  Failures: a lost miner's
// unfinished jobs go back to the front of their requests' queues unless a copy is out;
// only the job it was computing counts toward that job's cap of MAX_REQUEUES, after
// which the request is abandoned and its client disconnected; a lost client's requests
// are dropped and late results ignored.  A Request is served only if
// 0 <= Lower <= Upper <= 2^64-1 and Data fits the engine; otherwise the client's
// connection is closed.  stdout is never written.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "gpuhash.h"  // GPUHASH_MAX_MSG only: the server never loads the engine
#include "lsp_native.h"

namespace {

using lspn::BtcMsg;

constexpr int kMaxRequeues = 3;
// defaults: bitcoin/server.py REF_RATE, MINER_DEPTH, COPIES, SLACK, SLACK_FRAC
constexpr double kRefRate = 34.6e9;
constexpr int kDefaultDepth = 3;
constexpr int kDefaultCopies = 3;
constexpr double kSlack = 0.1;
constexpr double kSlackFrac = 0.25;

// GPU work of one MI355X for one LSP epoch (datagrams sent once), or for half a second or
// one epoch if shorter (sent in copies), to a power of two (server.py default_job_size)
uint64_t default_job_size(double epoch_s, int send_copies) {
    const double secs = send_copies <= 1 ? epoch_s : std::min(epoch_s, 0.5);
    long b = std::lround(std::log2(std::max(1.0, kRefRate * secs)));
    return 1ull << std::min(40L, std::max(30L, b));
}

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

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A range of one request.  The same Job sits in the queue of every miner holding a copy of
// it (speculative copies); `done` once any copy answered (bitcoin/server.py Job).
struct Job {
    uint64_t req, lo, hi;
    int requeues = 0;   // losses of a miner that was computing this job
    double sent = 0.0;  // first dispatch
    bool done = false;
    std::map<long long, double> holders;  // miner -> when its copy was sent
    double size() const { return (double)(hi - lo) + 1.0; }
};
using JobP = std::shared_ptr<Job>;

// Work and time of a miner's recent jobs, halved at each new result (server.py MinerRate).
struct MinerRate {
    double work = 0.0, secs = 0.0;
    void add(double n, double dt) {
        work = 0.5 * work + n;
        secs = 0.5 * secs + std::max(dt, 1e-6);
    }
    double rate() const { return work / secs; }
};

struct Request {
    uint64_t id;
    long long client;
    std::string data;
    uint64_t next_lo, upper;
    bool cut_all = false;  // every nonce is in some job (next_lo cannot pass 2^64-1)
    std::deque<JobP> requeued;
    int inflight = 0;
    bool has_best = false;
    uint64_t bh = 0, bn = 0;

    bool has_pending() const { return !requeued.empty() || !cut_all; }
    // nonces not yet handed to a miner (up to 2^64: hence 128 bits)
    unsigned __int128 remaining() const {
        unsigned __int128 n = cut_all ? 0 : (unsigned __int128)upper - next_lo + 1;
        for (const JobP& j : requeued) n += (unsigned __int128)j->hi - j->lo + 1;
        return n;
    }
    // a requeued job, else the next `size` nonces -- or all that is left when less than a
    // quarter job would remain (server.py Request.pop_job)
    JobP pop_job(uint64_t size) {
        if (!requeued.empty()) {
            JobP j = requeued.front();
            requeued.pop_front();
            return j;
        }
        const uint64_t lo = next_lo;
        const unsigned __int128 left = (unsigned __int128)upper - lo + 1;
        const uint64_t hi = left < (unsigned __int128)size + size / 4 ? upper : lo + (size - 1);
        if (hi == upper) cut_all = true;
        else next_lo = hi + 1;
        auto j = std::make_shared<Job>();
        j->req = id;
        j->lo = lo;
        j->hi = hi;
        return j;
    }
};

// bitcoin/server.py's Scheduler: depth, speculative copies (hedge "overdue"), the requeue
// cap charged to the job a lost miner was computing.
class Scheduler {
   public:
    Scheduler(uint64_t job_size, int depth, int copies, double slack, double slack_frac)
        : job_size_(job_size), depth_(depth < 1 ? 1 : depth), copies_(copies < 1 ? 1 : copies),
          slack_(slack), slack_frac_(slack_frac) {}

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
    bool next_assignment(long long& miner, JobP& job, std::string& data) {
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
        if (!r) return speculate(miner, job, data);
        job = r->pop_job(job_size_);
        job->sent = now_s();
        job->holders[best_m] = job->sent;
        r->inflight++;
        miners_[best_m].push_back(job);
        turn_[best_m] = tick_++;
        miner = best_m;
        data = r->data;
        return true;
    }

    // when next_assignment() may hand out a copy without any message arriving (< 0: never)
    double next_wakeup() {
        if (copies_ <= 1) return -1.0;
        bool idle = false;
        for (auto& [m, q] : miners_) idle = idle || q.empty();
        if (!idle) return -1.0;
        for (auto& [id, r] : requests_)
            if (r.has_pending()) return -1.0;
        double best = -1.0;
        for (const JobP& j : unfinished()) {
            if ((int)j->holders.size() >= copies_) continue;
            const double t = overdue_at(*j);
            if (t >= 0.0 && (best < 0.0 || t < best)) best = t;
        }
        return best;
    }

    // folds a miner's Result (its oldest job); true with the client and answer when done
    bool result(long long miner, uint64_t h, uint64_t n, long long& client, uint64_t& bh, uint64_t& bn) {
        auto it = miners_.find(miner);
        if (it == miners_.end() || it->second.empty()) return false;
        JobP job = it->second.front();
        it->second.pop_front();
        const double now = now_s();
        double sent = job->sent;
        auto hs = job->holders.find(miner);
        if (hs != job->holders.end()) {
            sent = hs->second;
            job->holders.erase(hs);
        }
        auto d = done_at_.find(miner);
        const double start = std::max(sent, d == done_at_.end() ? sent : d->second);
        done_at_[miner] = now;
        rates_[miner].add(job->size(), now - start);
        if (job->done) return false;  // another copy answered first
        job->done = true;
        auto r = requests_.find(job->req);
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

    // a lost miner's unfinished jobs go back to the front of their requests' queues unless
    // another miner holds a copy; only the job it was computing (its oldest) is charged
    // toward the requeue cap (server.py Scheduler.lost)
    void lost(long long conn) {
        auto it = miners_.find(conn);
        if (it != miners_.end()) {
            std::deque<JobP> jobs = std::move(it->second);
            miners_.erase(it);
            turn_.erase(conn);
            rates_.erase(conn);
            done_at_.erase(conn);
            logf("miner %lld lost", conn);
            const JobP current = jobs.empty() ? nullptr : jobs.front();
            for (auto jt = jobs.rbegin(); jt != jobs.rend(); ++jt) {  // oldest ends up first
                const JobP& j = *jt;
                j->holders.erase(conn);
                auto r = requests_.find(j->req);
                if (j->done || r == requests_.end()) continue;
                if (j == current && ++j->requeues > kMaxRequeues) {
                    logf("job [%llu, %llu] lost %d miners: request %llu abandoned, client %lld disconnected",
                         (unsigned long long)j->lo, (unsigned long long)j->hi, j->requeues,
                         (unsigned long long)j->req, r->second.client);
                    abandoned.push_back(r->second.client);
                    requests_.erase(r);
                    continue;
                }
                if (!j->holders.empty()) {
                    logf("job [%llu, %llu] of request %llu still held by %zu miner(s)", (unsigned long long)j->lo,
                         (unsigned long long)j->hi, (unsigned long long)j->req, j->holders.size());
                    continue;
                }
                r->second.inflight--;
                r->second.requeued.push_front(j);
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

    long long speculated() const { return speculated_; }

   private:
    uint64_t job_size_;
    int depth_, copies_;
    double slack_, slack_frac_;
    uint64_t next_id_ = 1, tick_ = 0;
    long long speculated_ = 0;
    std::map<uint64_t, Request> requests_;
    std::map<long long, std::deque<JobP>> miners_;
    std::map<long long, uint64_t> turn_;
    std::map<long long, MinerRate> rates_;
    std::map<long long, double> done_at_;

    // a miner's learned rate, a new miner's the median of the known ones (< 0: none known)
    double rate(long long miner) const {
        auto it = rates_.find(miner);
        if (it != rates_.end()) return it->second.rate();
        std::vector<double> known;
        for (auto& [m, r] : rates_) known.push_back(r.rate());
        if (known.empty()) return -1.0;
        std::sort(known.begin(), known.end());
        return known[known.size() / 2];
    }

    // when `miner`'s Result for `job` is due plus the slack (< 0: unknown)
    double expected(const Job& job, long long miner) const {
        const double rt = rate(miner);
        if (rt <= 0.0) return -1.0;
        auto d = done_at_.find(miner);
        double t = d == done_at_.end() ? 0.0 : d->second;
        auto q = miners_.find(miner);
        if (q == miners_.end()) return -1.0;
        for (const JobP& j : q->second) {
            auto h = j->holders.find(miner);
            t = std::max(t, h == j->holders.end() ? j->sent : h->second) + j->size() / rt;
            if (j.get() == &job) return t + std::max(slack_, slack_frac_ * j->size() / rt);
        }
        return -1.0;
    }

    // when every copy of `job` is overdue (< 0: some holder's rate is unknown)
    double overdue_at(const Job& job) const {
        double worst = -1.0;
        for (auto& [m, sent] : job.holders) {
            const double t = expected(job, m);
            if (t < 0.0) return -1.0;
            worst = std::max(worst, t);
        }
        return worst;
    }

    std::vector<JobP> unfinished() const {
        std::vector<JobP> out;
        for (auto& [m, q] : miners_)
            for (const JobP& j : q)
                if (!j->done && requests_.count(j->req) && std::find(out.begin(), out.end(), j) == out.end())
                    out.push_back(j);
        return out;
    }

    bool speculate(long long& miner, JobP& job, std::string& data) {
        if (copies_ <= 1) return false;
        long long idle = 0;
        bool any = false;
        double idle_rate = 0.0;
        for (auto& [m, q] : miners_) {
            if (!q.empty()) continue;
            const double rt = std::max(0.0, rate(m));
            if (!any || rt > idle_rate || (rt == idle_rate && turn_.at(m) < turn_.at(idle))) {
                idle = m;
                idle_rate = rt;
                any = true;
            }
        }
        if (!any) return false;
        const double now = now_s();
        JobP best;
        double best_t = 0.0;
        for (const JobP& j : unfinished()) {
            if ((int)j->holders.size() >= copies_) continue;
            const double t = overdue_at(*j);
            if (t < 0.0 || t > now) continue;
            if (!best || t < best_t || (t == best_t && j->sent < best->sent)) {
                best = j;
                best_t = t;
            }
        }
        if (!best) return false;
        logf("copy of job [%llu, %llu] of request %llu to miner %lld (held by %zu miner(s), overdue)",
             (unsigned long long)best->lo, (unsigned long long)best->hi, (unsigned long long)best->req, idle,
             best->holders.size());
        best->holders[idle] = now;
        miners_[idle].push_back(best);
        turn_[idle] = tick_++;
        speculated_++;
        miner = idle;
        job = best;
        data = requests_.at(best->req).data;
        return true;
    }
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
    const char* backup = std::getenv("GPUHASH_BACKUP");
    const int copies = backup && std::strcmp(backup, "0") == 0 ? 1 : (int)env_u64("GPUHASH_COPIES", kDefaultCopies);
    Scheduler sched(env_u64("GPUHASH_JOB_SIZE", default_job_size(params.epoch_ms / 1000.0, params.send_copies)),
                    (int)env_u64("GPUHASH_MINER_DEPTH", kDefaultDepth),
                    copies, kSlack, kSlackFrac);
    // the configuration, in the words of server.py's serve() (tests compare the two)
    logf("config: jobs of %llu nonces, depth %d, %d live copies of an overdue job; LSP epoch %d ms, limit %d, "
         "window %d, send copies %d",
         (unsigned long long)env_u64("GPUHASH_JOB_SIZE", default_job_size(params.epoch_ms / 1000.0, params.send_copies)),
         (int)env_u64("GPUHASH_MINER_DEPTH", kDefaultDepth), copies, params.epoch_ms, params.epoch_limit,
         params.window, params.send_copies);

    auto dispatch = [&] {
        while (!sched.abandoned.empty()) {
            srv.close_conn(sched.abandoned.front());
            sched.abandoned.pop_front();
        }
        long long miner;
        JobP job;
        std::string data;
        while (sched.next_assignment(miner, job, data)) {
            BtcMsg req;
            req.type = lspn::Request;
            req.data = data;
            req.lower = job->lo;
            req.upper = job->hi;
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
        // wake for the scheduler's own timer (the next job to become overdue) as for a message
        const double wake = sched.next_wakeup();
        lspn::Server::Event e = wake < 0.0 ? srv.read() : srv.read_until(wake);
        if (e.timed_out) {
            dispatch();
            continue;
        }
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
