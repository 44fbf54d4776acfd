// rate_limiting.cpp -- limiter classes over the tbe C ABI (see rate_limiting.hpp).
//
// Every limiter owns a detail::LimiterCore: one engine (tbe_create), a string-key
// directory for the partitioned limiters (PTB:42 BucketId = InstanceName + resourceID),
// and one submitter thread.  Callers enqueue requests; the submitter takes the longest
// run of same-mode requests at the head of the queue (up to MaxBatch) and makes ONE
// engine call for it, then completes the callers' futures.  Commands (replenish ticks,
// state queries, dispose) go through the same queue, so every engine call happens on one
// thread (the ABI is not re-entrant) in arrival order -- the order Redis serialises the
// scripts in.  Requests are time-stamped on arrival with the limiter's TimeSource, which
// plays Redis TIME (TB:202).
#include "rate_limiting.hpp"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <shared_mutex>
#include <thread>
#include <unordered_set>
#include <variant>

namespace tbe::rate_limiting {

// ------------------------------------------------------------------ value types
TimeSpan TimeSpan::FromSeconds(double s) {
    // .NET 7 TimeSpan.Interval: ticks = value * scale, truncated toward zero; overflow throws.
    if (std::isnan(s)) throw ArgumentException("TimeSpan does not accept floating point Not-a-Number values.", "value");
    const double t = s * (double)TicksPerSecond;
    if (t >= 9223372036854775807.0 || t < -9223372036854775808.0)
        throw std::overflow_error("TimeSpan overflowed because the duration is too long.");
    return TimeSpan{(int64_t)t};
}

static std::string format_timespan(TimeSpan ts) {  // TimeSpan.ToString() ("c" format)
    int64_t t = ts.ticks;
    std::string out;
    if (t < 0) {
        out = "-";
        t = -t;
    }
    const int64_t days = t / (TimeSpan::TicksPerSecond * 86400);
    int64_t rem = t % (TimeSpan::TicksPerSecond * 86400);
    const int64_t h = rem / (TimeSpan::TicksPerSecond * 3600);
    rem %= TimeSpan::TicksPerSecond * 3600;
    const int64_t m = rem / (TimeSpan::TicksPerSecond * 60);
    rem %= TimeSpan::TicksPerSecond * 60;
    const int64_t sec = rem / TimeSpan::TicksPerSecond;
    const int64_t frac = rem % TimeSpan::TicksPerSecond;
    char buf[64];
    if (days) {
        std::snprintf(buf, sizeof buf, "%lld.", (long long)days);
        out += buf;
    }
    std::snprintf(buf, sizeof buf, "%02lld:%02lld:%02lld", (long long)h, (long long)m, (long long)sec);
    out += buf;
    if (frac) {
        std::snprintf(buf, sizeof buf, ".%07lld", (long long)frac);
        out += buf;
    }
    return out;
}

std::vector<std::string> RateLimitLease::MetadataNames() const { return {"RETRY_AFTER"}; }

bool RateLimitLease::TryGetRetryAfter(TimeSpan &out) const {
    if (!retry_after_) return false;
    out = *retry_after_;
    return true;
}

std::string RateLimitLease::ToString() const {
    std::string s = std::string("Lease IsAcquired: ") + (acquired_ ? "True" : "False");
    if (retry_after_) s += " RETRY_AFTER: " + format_timespan(*retry_after_);
    return s;
}

int64_t SystemClockMicros() {
    using namespace std::chrono;
    return duration_cast<microseconds>(system_clock::now().time_since_epoch()).count();
}

double RedisTokenBucketRateLimiterOptions::FillRatePerSecond() const {
    return tbe_fill_rate(TokensPerPeriod, ReplenishmentPeriod.ticks);  // TBO:82-85
}

RateLimitLease RateLimiter::AttemptAcquire(int permitCount) {
    if (permitCount < 0) throw ArgumentOutOfRangeException("permitCount must be >= 0", "permitCount");
    return AttemptAcquireCore(permitCount);
}

std::future<RateLimitLease> RateLimiter::AcquireAsync(int permitCount, CancellationToken ct) {
    if (permitCount < 0) throw ArgumentOutOfRangeException("permitCount must be >= 0", "permitCount");
    return AcquireAsyncCore(permitCount, ct);
}

bool CancellationToken::IsCancellationRequested() const {
    if (!s_) return false;
    std::lock_guard<std::mutex> g(s_->mu);
    return s_->canceled;
}

uint64_t CancellationToken::Register(std::function<void()> fn) const {
    if (!s_) return 0;
    {
        std::lock_guard<std::mutex> g(s_->mu);
        if (!s_->canceled) {
            const uint64_t h = s_->next++;
            s_->callbacks.emplace(h, std::move(fn));
            return h;
        }
    }
    fn();  // already canceled: run at once, as CancellationToken.Register does
    return 0;
}

void CancellationToken::Unregister(uint64_t handle) const {
    if (!s_ || !handle) return;
    std::lock_guard<std::mutex> g(s_->mu);
    s_->callbacks.erase(handle);
}

size_t CancellationToken::RegisteredCount() const {
    if (!s_) return 0;
    std::lock_guard<std::mutex> g(s_->mu);
    return s_->callbacks.size();
}

void CancellationTokenSource::Cancel() {
    std::map<uint64_t, std::function<void()>> fns;
    {
        std::lock_guard<std::mutex> g(s_->mu);
        if (s_->canceled) return;
        s_->canceled = true;
        fns.swap(s_->callbacks);
    }
    for (auto &f : fns) f.second();
}

// ------------------------------------------------------------------ the core
namespace detail {

class LimiterCore {
public:
    LimiterCore(tbe_kind kind, const RedisQueueingTokenBucketRateLimiterOptions &o, bool partitioned,
                const char *type_name)
        : kind_(kind), opt_(o), partitioned_(partitioned), type_name_(type_name) {
        // Constructor checks in reference order (TB:24-42; A:44-72).
        if (o.TokenLimit <= 0 || o.TokensPerPeriod <= 0)
            throw ArgumentException("Both TokenLimit and TokensPerPeriod must be set to values greater than 0.",
                                    "options");
        if (kind != TBE_KIND_TOKEN_BUCKET && o.QueueLimit < 0)
            throw ArgumentException("QueueLimit must be set to a value greater than or equal to 0.", "options");
        if (o.ReplenishmentPeriod.ticks < 0)
            throw ArgumentException("ReplenishmentPeriod must be set to a value greater than or equal to TimeSpan.Zero.",
                                    "options");
        if (partitioned && o.PartitionLimit == 0)
            throw ArgumentException("PartitionLimit must be greater than 0.", "options");
        if (o.MaxBatch == 0) throw ArgumentException("MaxBatch must be greater than 0.", "options");
        clock_ = o.TimeSource ? o.TimeSource : Clock(SystemClockMicros);
        tbe_config c{};
        c.struct_size = sizeof c;
        c.kind = kind;
        c.n_keys = partitioned ? o.PartitionLimit : 1;
        c.token_limit = o.TokenLimit;
        c.tokens_per_period = o.TokensPerPeriod;
        c.replenishment_period_ticks = o.ReplenishmentPeriod.ticks;
        c.queue_limit = kind == TBE_KIND_TOKEN_BUCKET ? 0 : o.QueueLimit;
        c.queue_order = (int32_t)o.QueueProcessingOrder;
        c.device = o.Device;
        c.max_batch = o.MaxBatch;
        c.zero_wait_slots = kind == TBE_KIND_APPROXIMATE ? o.ZeroWaitSlots : 0;
        const tbe_status st = tbe_create(&c, &eng_);
        if (st == TBE_EINVAL) throw ArgumentException(std::string("invalid limiter options: ") + tbe_last_error(nullptr), "options");
        if (st != TBE_OK) throw RateLimiterEngineException(st, std::string("tbe_create failed: ") + tbe_last_error(nullptr));
        inbox_->core = this;
        submitter_ = std::thread([this] { Loop(); });
        if (kind != TBE_KIND_TOKEN_BUCKET && o.AutoReplenishment && o.ReplenishmentPeriod.ticks > 0)
            timer_ = std::thread([this] { TimerLoop(); });
    }

    ~LimiterCore() { Dispose(); }

    const RedisQueueingTokenBucketRateLimiterOptions &options() const { return opt_; }

    // InstanceName + resourceID -> dense key (PTB:42).  Exact strings, never hashed.
    // When all PartitionLimit keys are taken, the keys whose Redis hash would have expired
    // (TB:232-235: EXPIRE after the last grant, or never granted) are reclaimed: their
    // bucket is absent, exactly what a new string's bucket is.  The directory lookup and
    // the enqueue happen under a shared lock that the reclaim takes exclusively, and keys
    // with requests still in the submitter's queue are kept, so no request of an old
    // string can land on a reassigned key.
    std::future<RateLimitLease> SubmitResource(const std::string &resource, int32_t permits, int mode) {
        for (int attempt = 0;; ++attempt) {
            {
                std::shared_lock<std::shared_mutex> g(reclaim_mu_);
                uint64_t k;
                if (TryKeyOf(resource, k)) return Submit(k, permits, mode);
            }
            if (attempt)
                throw RateLimiterEngineException(TBE_ERANGE, "PartitionLimit reached: no key left for '" +
                                                                 opt_.InstanceName + resource + "'");
            ThrowIfDisposed();
            Run([this] { Reclaim(); });
        }
    }

    bool TryKeyOf(const std::string &resource, uint64_t &key) {
        const std::string bucket = opt_.InstanceName + resource;
        std::lock_guard<std::mutex> g(dir_mu_);
        auto it = dir_.find(bucket);
        if (it != dir_.end()) {
            key = it->second;
            return true;
        }
        if (!free_ids_.empty()) {
            key = free_ids_.back();
            free_ids_.pop_back();
        } else if (names_.size() < opt_.PartitionLimit) {
            key = names_.size();
            names_.emplace_back();
        } else {
            return false;
        }
        names_[key] = bucket;
        dir_.emplace(bucket, key);
        return true;
    }

    // Submitter thread (so every request enqueued before it has been decided).
    uint64_t Reclaim() {
        std::unique_lock<std::shared_mutex> x(reclaim_mu_);
        std::unordered_set<uint64_t> busy;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (auto &v : q_)
                if (auto *r = std::get_if<Req>(&v)) busy.insert(r->key);
        }
        std::lock_guard<std::mutex> g(dir_mu_);
        const uint64_t n = names_.size();
        if (n == 0) return 0;
        // TB:234: EXPIRE ceil(min(max(capacity / fill_rate, 1), 31536000)) seconds; the
        // engine's expiry test is tbe_query's (millisecond resolution).
        double q = (double)opt_.TokenLimit / opt_.FillRatePerSecond();
        q = (1.0 > q) ? 1.0 : q;
        q = (31536000.0 < q) ? 31536000.0 : q;
        const int64_t ttl_ms = (int64_t)std::ceil(q) * 1000;
        const int64_t now_ms = clock_() / 1000;
        std::vector<uint8_t> is_free(n, 0);
        for (uint64_t k : free_ids_) is_free[k] = 1;
        uint64_t freed = 0;
        // the table is read back in chunks (bounded host memory); a freed key's row is
        // then written back absent, so a new string starts from a full bucket whatever
        // the clock does later (a system clock may step backwards)
        constexpr uint64_t kChunk = 1u << 20;
        std::vector<double> v(std::min(n, kChunk));
        std::vector<int64_t> t(std::min(n, kChunk));
        for (uint64_t k0 = 0; k0 < n; k0 += kChunk) {
            const uint64_t m = std::min(kChunk, n - k0);
            Check(tbe_export_state(eng_, k0, m, v.data(), t.data()));
            bool cleared = false;
            for (uint64_t j = 0; j < m; ++j) {
                const uint64_t k = k0 + j;
                if (is_free[k] || busy.count(k)) continue;
                if (t[j] != INT64_MIN && now_ms <= t[j] / 1000 + ttl_ms) continue;  // still present
                dir_.erase(names_[k]);
                names_[k].clear();
                last_reply_.erase(k);
                free_ids_.push_back(k);
                if (t[j] != INT64_MIN) {
                    t[j] = INT64_MIN;
                    cleared = true;
                }
                ++freed;
            }
            // this thread is the engine's only submitter: the other rows go back unchanged
            if (cleared) Check(tbe_import_state(eng_, k0, m, v.data(), t.data()));
        }
        reclaimed_ += freed;
        return freed;
    }

    uint64_t Reclaimed() const { return reclaimed_.load(); }

    bool KnownKey(const std::string &resource, uint64_t &key) {
        std::lock_guard<std::mutex> g(dir_mu_);
        auto it = dir_.find(opt_.InstanceName + resource);
        if (it == dir_.end()) return false;
        key = it->second;
        return true;
    }

    void ThrowIfDisposed() const {
        if (disposed_.load()) throw ObjectDisposedException(type_name_);
    }

    std::future<RateLimitLease> Submit(uint64_t key, int32_t permits, int mode,
                                       const CancellationToken &ct = {}) {
        Req r;
        r.key = key;
        r.permits = permits;
        r.mode = mode;
        r.ct = ct;
        std::future<RateLimitLease> f = r.done.get_future();
        {
            std::lock_guard<std::mutex> g(mu_);
            if (disposed_.load()) throw ObjectDisposedException(type_name_);
            r.ts = clock_();
            q_.emplace_back(std::move(r));
        }
        cv_.notify_one();
        return f;
    }

    // Run fn on the submitter thread, between batches, and wait for it.
    template <class F>
    auto Run(F &&fn) -> decltype(fn()) {
        using R = decltype(fn());
        auto task = std::make_shared<std::packaged_task<R()>>(std::forward<F>(fn));
        std::future<R> f = task->get_future();
        {
            std::lock_guard<std::mutex> g(mu_);
            if (stop_) throw ObjectDisposedException(type_name_);
            q_.emplace_back(Cmd{[task] { (*task)(); }});
        }
        cv_.notify_one();
        return f.get();
    }

    // ---- state readers (on the submitter thread via Run)
    int EstimatedRemaining() const { return estimated_.load(); }

    int LastReply(uint64_t key) {
        std::lock_guard<std::mutex> g(dir_mu_);
        auto it = last_reply_.find(key);
        return it == last_reply_.end() ? opt_.TokenLimit : it->second;
    }

    struct ApproxState {
        int32_t local = 0, global = 0, available = 0;
        double est = 1.0;
        uint32_t queued = 0;
        int64_t queued_permits = 0;
    };
    ApproxState QueryApprox(uint64_t key) {  // submitter thread only
        ApproxState s;
        Check(tbe_approx_query(eng_, key, &s.local, &s.global, &s.est, &s.available, &s.queued));
        if (s.queued) {
            std::vector<int64_t> ids(s.queued);
            std::vector<int32_t> ps(s.queued);
            uint32_t cnt = 0;
            Check(tbe_queue_of(eng_, key, ids.data(), ps.data(), s.queued, &cnt));
            for (uint32_t j = 0; j < cnt && j < s.queued; ++j) s.queued_permits += ps[j];
        }
        return s;
    }

    // One replenish tick (Q:237-271) / RefreshAsync (A:412-508), on the submitter thread.
    void RefreshNow() {
        if (disposed_.load()) return;  // A:414-417
        const int64_t now = clock_();
        uint64_t n = 0;
        if (kind_ == TBE_KIND_QUEUEING)
            Check(tbe_refresh(eng_, now, &n));
        else
            Check(tbe_approx_refresh(eng_, now, &n));
        if (n) {
            std::vector<uint64_t> keys(n);
            std::vector<int64_t> ids(n);
            std::vector<int32_t> rem(n);
            uint64_t w = 0;
            Check(tbe_refresh_log(eng_, keys.data(), ids.data(), rem.data(), n, &w));
            for (uint64_t i = 0; i < w; ++i) {
                if (!Complete(ids[i], RateLimitLease(true))) continue;
                if (kind_ == TBE_KIND_QUEUEING) Remember(keys[i], rem[i]);
            }
        }
        if (kind_ == TBE_KIND_APPROXIMATE && !partitioned_) {  // A:503-506
            const ApproxState s = QueryApprox(0);
            if ((int32_t)((uint32_t)s.global + (uint32_t)s.local) == 0)
                idle_since_ns_.store(SteadyNs());
        }
    }

    std::optional<TimeSpan> IdleDuration() const {
        const int64_t since = idle_since_ns_.load();
        if (since < 0) return std::nullopt;
        return TimeSpan{(SteadyNs() - since) / 100};
    }

    // Dispose (TB:85-94; A:274-300): fail every queued request, stop, free the device.
    void Dispose() {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (disposed_.exchange(true)) return;
        }
        {  // later cancellations find nothing to cancel: dispose fails the queue below
            std::lock_guard<std::mutex> g(inbox_->mu);
            inbox_->closed = true;
        }
        {
            std::lock_guard<std::mutex> g(timer_mu_);
            timer_stop_ = true;
        }
        timer_cv_.notify_all();
        if (timer_.joinable()) timer_.join();
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.emplace_back(Cmd{[this] {
                for (auto &w : waiting_) {
                    w.second.ct.Unregister(w.second.reg);
                    w.second.done.set_value(RateLimitLease(false));
                }
                waiting_.clear();
            }});
            stop_ = true;
        }
        cv_.notify_one();
        if (submitter_.joinable()) submitter_.join();
        tbe_destroy(eng_);
        eng_ = nullptr;
    }

private:
    struct Req {
        uint64_t key = 0;
        int32_t permits = 0;
        int64_t ts = 0;
        int mode = 0;
        CancellationToken ct;
        std::promise<RateLimitLease> done;
    };
    struct Cmd {
        std::function<void()> fn;
    };
    // Cancellations of queued requests (CancelQueueState.TrySetCanceled, Q:480-506,
    // A:531-557) arrive on whatever thread cancels the token; they wait here for the
    // submitter, which applies them with one tbe_queue_cancel call before its next batch.
    // Token callbacks hold the inbox, not the core, so they outlive a disposed limiter.
    struct CancelInbox {
        std::mutex mu;
        bool closed = false;
        LimiterCore *core = nullptr;
        std::vector<std::pair<uint64_t, int64_t>> pending;  // (key, request id)
        void Post(uint64_t key, int64_t id) {
            std::lock_guard<std::mutex> g(mu);
            if (closed) return;
            pending.emplace_back(key, id);
            core->WakeForCancel();
        }
    };

    void WakeForCancel() {
        {
            std::lock_guard<std::mutex> g(mu_);
            cancel_wake_ = true;
        }
        cv_.notify_one();
    }

    void FlushCancels() {  // submitter thread
        std::vector<std::pair<uint64_t, int64_t>> list;
        {
            std::lock_guard<std::mutex> g(inbox_->mu);
            list.swap(inbox_->pending);
        }
        if (list.empty()) return;
        const uint64_t n = list.size();
        std::vector<uint64_t> keys(n);
        std::vector<int64_t> ids(n);
        std::vector<uint8_t> hit(n);
        for (uint64_t i = 0; i < n; ++i) {
            keys[i] = list[i].first;
            ids[i] = list[i].second;
        }
        uint64_t m = 0;
        if (tbe_queue_cancel(eng_, keys.data(), ids.data(), n, hit.data(), &m) != TBE_OK) {
            // keep them: the next flush retries (the engine error also surfaces on the next batch)
            std::lock_guard<std::mutex> g(inbox_->mu);
            list.insert(list.end(), inbox_->pending.begin(), inbox_->pending.end());
            inbox_->pending.swap(list);
            return;
        }
        for (uint64_t i = 0; i < n; ++i) {
            if (!hit[i]) continue;  // already completed: TrySetCanceled returns false
            auto it = waiting_.find(ids[i]);
            if (it == waiting_.end()) continue;
            it->second.done.set_exception(std::make_exception_ptr(OperationCanceledException()));
            waiting_.erase(it);   // its callback has run: nothing left registered
        }
    }

    static int64_t SteadyNs() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }

    void Check(tbe_status st) {
        if (st != TBE_OK) throw RateLimiterEngineException(st, tbe_last_error(eng_));
    }

    void Remember(uint64_t key, int32_t rem) {  // TB:73 _estimatedRemainingPermits = result[1]
        if (rem < 0) return;
        estimated_.store(rem);
        if (partitioned_) {
            std::lock_guard<std::mutex> g(dir_mu_);
            last_reply_[key] = rem;
        }
    }

    void Loop() {
        std::vector<Req> batch;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !q_.empty() || stop_ || cancel_wake_; });
            if (cancel_wake_) {
                cancel_wake_ = false;
                lk.unlock();
                FlushCancels();
                continue;
            }
            if (q_.empty()) break;  // stop_ and drained
            if (auto *c = std::get_if<Cmd>(&q_.front())) {
                std::function<void()> fn = std::move(c->fn);
                q_.pop_front();
                lk.unlock();
                fn();
                continue;
            }
            const int mode = std::get<Req>(q_.front()).mode;
            batch.clear();
            while (!q_.empty() && batch.size() < opt_.MaxBatch) {
                Req *r = std::get_if<Req>(&q_.front());
                if (!r || r->mode != mode) break;
                const bool precanceled = r->ct.IsCancellationRequested();
                batch.push_back(std::move(*r));
                q_.pop_front();
                // A token canceled before the call cancels the request as soon as it queues
                // (Register runs the callback at once, A:169-175): end the batch here so the
                // cancel lands before the next request of the key is decided.
                if (precanceled && mode != kTbAcquire) break;
            }
            lk.unlock();
            try {
                RunBatch(mode, batch);
            } catch (...) {  // engine error: every caller of the batch sees it (TB:63 propagation)
                for (auto &r : batch) {
                    try {
                        r.done.set_exception(std::current_exception());
                    } catch (const std::future_error &) {
                    }
                }
            }
        }
    }

    void RunBatch(int mode, std::vector<Req> &batch) {
        const uint64_t n = batch.size();
        keys_.resize(n);
        permits_.resize(n);
        ts_.resize(n);
        status_.resize(n);
        rem_.resize(n);
        for (uint64_t i = 0; i < n; ++i) {
            keys_[i] = batch[i].key;
            permits_[i] = batch[i].permits;
            ts_[i] = batch[i].ts;
        }
        uint64_t n_ev = 0;
        const int64_t id_base = next_id_;
        switch (mode) {
        case kTbAcquire:
            Check(tbe_acquire_batch(eng_, keys_.data(), permits_.data(), ts_.data(), n, status_.data(), rem_.data()));
            break;
        case kQueueWait:
            Check(tbe_wait_batch(eng_, keys_.data(), permits_.data(), ts_.data(), n, id_base, status_.data(),
                                 rem_.data(), &n_ev));
            next_id_ += (int64_t)n;
            break;
        case kQueueAttempt:
            Check(tbe_queue_attempt_batch(eng_, keys_.data(), permits_.data(), ts_.data(), n, status_.data(),
                                          rem_.data()));
            break;
        default:  // kApproxWait / kApproxAttempt
            Check(tbe_approx_acquire_batch(eng_, keys_.data(), permits_.data(), n, mode == kApproxWait ? 1 : 0,
                                           id_base, status_.data(), rem_.data(), &n_ev));
            next_id_ += (int64_t)n;
            break;
        }
        if (opt_.OnBatch)
            opt_.OnBatch(BatchTrace{mode, n, keys_.data(), permits_.data(), ts_.data(), status_.data(), rem_.data()});

        // Approximate failed leases carry RetryAfter (A:390-395), from the key's state after
        // this micro-batch: deficit = max(0, consumed + p + queued permits - TokenLimit).
        std::unordered_map<uint64_t, ApproxState> approx;
        for (uint64_t i = 0; i < n; ++i) {
            Req &r = batch[i];
            const uint8_t s = status_[i];
            if (mode == kTbAcquire) {
                Remember(r.key, rem_[i]);
                r.done.set_value(RateLimitLease(s != 0));
                continue;
            }
            if (mode == kQueueWait || mode == kQueueAttempt) Remember(r.key, rem_[i]);
            if (s == TBE_WAIT_GRANTED) {
                if (mode == kApproxWait || mode == kApproxAttempt) idle_since_ns_.store(-1);  // A:204
                r.done.set_value(RateLimitLease(true));
            } else if (s == TBE_WAIT_QUEUED) {
                const int64_t id = id_base + (int64_t)i;
                Waiter &wt = waiting_.emplace(id, Waiter{std::move(r.done), r.ct, 0}).first->second;
                if (r.ct.CanBeCanceled()) {  // A:166-175
                    std::shared_ptr<CancelInbox> box = inbox_;
                    const uint64_t key = r.key;
                    wt.reg = r.ct.Register([box, key, id] { box->Post(key, id); });
                }
            } else if (mode == kApproxWait || mode == kApproxAttempt) {
                auto it = approx.find(r.key);
                if (it == approx.end()) it = approx.emplace(r.key, QueryApprox(r.key)).first;
                const ApproxState &a = it->second;
                const int64_t consumed = (int32_t)((uint32_t)a.global + (uint32_t)a.local);
                const int64_t deficit = std::max<int64_t>(0, consumed + r.permits + a.queued_permits - opt_.TokenLimit);
                r.done.set_value(RateLimitLease(false, TimeSpan::FromSeconds((double)deficit * opt_.FillRatePerSecond())));
            } else {
                r.done.set_value(RateLimitLease(false));
            }
        }
        if (n_ev) {  // NewestFirst evictions complete with FailedLease (Q:94-109, A:146-157)
            std::vector<uint64_t> cause(n_ev);
            std::vector<int64_t> ids(n_ev);
            uint64_t w = 0;
            Check(tbe_evicted(eng_, cause.data(), ids.data(), n_ev, &w));
            for (uint64_t j = 0; j < w; ++j) Complete(ids[j], RateLimitLease(false));
        }
    }

    void TimerLoop() {  // the reference's Timer(Refresh, ..., period, period) (A:77)
        const auto period = std::chrono::nanoseconds(opt_.ReplenishmentPeriod.ticks * 100);
        std::unique_lock<std::mutex> lk(timer_mu_);
        for (;;) {
            if (timer_cv_.wait_for(lk, period, [&] { return timer_stop_; })) return;
            // Start a refresh only if the previous one has completed (A:402-409).
            if (refresh_pending_.exchange(true)) continue;
            std::lock_guard<std::mutex> g(mu_);
            if (stop_) return;
            q_.emplace_back(Cmd{[this] {
                try {
                    RefreshNow();
                } catch (...) {  // the reference logs and carries on (A:445-449)
                }
                refresh_pending_.store(false);
            }});
            cv_.notify_one();
        }
    }

    tbe_kind kind_;
    RedisQueueingTokenBucketRateLimiterOptions opt_;
    bool partitioned_;
    const char *type_name_;
    Clock clock_;
    tbe_engine *eng_ = nullptr;

    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::variant<Req, Cmd>> q_;
    bool stop_ = false;
    bool cancel_wake_ = false;  // under mu_
    std::shared_ptr<CancelInbox> inbox_ = std::make_shared<CancelInbox>();
    std::atomic<bool> disposed_{false};
    std::thread submitter_;

    std::mutex timer_mu_;
    std::condition_variable timer_cv_;
    bool timer_stop_ = false;
    std::atomic<bool> refresh_pending_{false};
    std::thread timer_;

    std::mutex dir_mu_;
    std::unordered_map<std::string, uint64_t> dir_;
    std::vector<std::string> names_;       // key -> bucket string
    std::vector<uint64_t> free_ids_;       // reclaimed keys, reused first
    std::shared_mutex reclaim_mu_;
    std::atomic<uint64_t> reclaimed_{0};
    std::unordered_map<uint64_t, int32_t> last_reply_;
    std::atomic<int> estimated_{0};
    std::atomic<int64_t> idle_since_ns_{-1};

    // submitter-thread state
    int64_t next_id_ = 0;
    // A queued request: its promise and its token registration, disposed when the request
    // completes (granted, evicted, failed at dispose) so a long-lived token does not keep
    // one callback per request it ever saw (CancellationTokenRegistration.Dispose, Q:263).
    struct Waiter {
        std::promise<RateLimitLease> done;
        CancellationToken ct;
        uint64_t reg;
    };
    std::unordered_map<int64_t, Waiter> waiting_;
    bool Complete(int64_t id, RateLimitLease lease) {
        auto it = waiting_.find(id);
        if (it == waiting_.end()) return false;
        it->second.ct.Unregister(it->second.reg);
        it->second.done.set_value(std::move(lease));
        waiting_.erase(it);
        return true;
    }
    std::vector<uint64_t> keys_;
    std::vector<int32_t> permits_;
    std::vector<int64_t> ts_;
    std::vector<uint8_t> status_;
    std::vector<int32_t> rem_;
};

static RedisQueueingTokenBucketRateLimiterOptions widen(const RedisTokenBucketRateLimiterOptions &o) {
    RedisQueueingTokenBucketRateLimiterOptions q;
    static_cast<RedisTokenBucketRateLimiterOptions &>(q) = o;
    return q;
}

}  // namespace detail

using detail::LimiterCore;

// ------------------------------------------------------------------ token bucket
RedisTokenBucketRateLimiter::RedisTokenBucketRateLimiter(const RedisTokenBucketRateLimiterOptions &o)
    : core_(std::make_unique<LimiterCore>(TBE_KIND_TOKEN_BUCKET, detail::widen(o), false,
                                          "RedisTokenBucketRateLimiter")) {}
RedisTokenBucketRateLimiter::~RedisTokenBucketRateLimiter() = default;
int RedisTokenBucketRateLimiter::GetAvailablePermits() { return core_->EstimatedRemaining(); }
RateLimitLease RedisTokenBucketRateLimiter::AttemptAcquireCore(int p) { return core_->Submit(0, p, kTbAcquire).get(); }
std::future<RateLimitLease> RedisTokenBucketRateLimiter::AcquireAsyncCore(int p, const CancellationToken &) {
    return core_->Submit(0, p, kTbAcquire);  // never queues: nothing to cancel (TB:58-82)
}
void RedisTokenBucketRateLimiter::DisposeCore() { core_->Dispose(); }

PartitionedRedisTokenBucketRateLimiter::PartitionedRedisTokenBucketRateLimiter(const RedisTokenBucketRateLimiterOptions &o)
    : core_(std::make_unique<LimiterCore>(TBE_KIND_TOKEN_BUCKET, detail::widen(o), true,
                                          "PartitionedRedisTokenBucketRateLimiter")) {}
PartitionedRedisTokenBucketRateLimiter::~PartitionedRedisTokenBucketRateLimiter() = default;
int PartitionedRedisTokenBucketRateLimiter::GetAvailablePermits(const std::string &id) {
    core_->ThrowIfDisposed();
    uint64_t k;
    return core_->KnownKey(id, k) ? core_->LastReply(k) : core_->options().TokenLimit;
}
RateLimitLease PartitionedRedisTokenBucketRateLimiter::AttemptAcquireCore(const std::string &id, int p) {
    core_->ThrowIfDisposed();
    return core_->SubmitResource(id, p, kTbAcquire).get();
}
std::future<RateLimitLease> PartitionedRedisTokenBucketRateLimiter::AcquireAsyncCore(const std::string &id, int p,
                                                                                     const CancellationToken &) {
    core_->ThrowIfDisposed();
    return core_->SubmitResource(id, p, kTbAcquire);
}
void PartitionedRedisTokenBucketRateLimiter::DisposeCore() { core_->Dispose(); }
uint64_t PartitionedRedisTokenBucketRateLimiter::ReclaimExpired() {
    core_->ThrowIfDisposed();
    return core_->Run([this] { return core_->Reclaim(); });
}

// ------------------------------------------------------------------ queueing
static void check_limit(int p, int limit) {  // Q:70-73, A:87-90, A:119-122
    if (p > limit)
        throw ArgumentOutOfRangeException(std::to_string(p) + " token(s) exceeds the token limit of " +
                                              std::to_string(limit), "permitCount");
}

RedisQueueingTokenBucketRateLimiter::RedisQueueingTokenBucketRateLimiter(const RedisQueueingTokenBucketRateLimiterOptions &o)
    : core_(std::make_unique<LimiterCore>(TBE_KIND_QUEUEING, o, false, "RedisQueueingTokenBucketRateLimiter")) {}
RedisQueueingTokenBucketRateLimiter::~RedisQueueingTokenBucketRateLimiter() = default;
int RedisQueueingTokenBucketRateLimiter::GetAvailablePermits() { return core_->EstimatedRemaining(); }
bool RedisQueueingTokenBucketRateLimiter::TryReplenish() {
    if (core_->options().AutoReplenishment) return false;
    core_->ThrowIfDisposed();
    core_->Run([this] { core_->RefreshNow(); });
    return true;
}
RateLimitLease RedisQueueingTokenBucketRateLimiter::AttemptAcquireCore(int p) {
    check_limit(p, core_->options().TokenLimit);
    return core_->Submit(0, p, kQueueAttempt).get();
}
std::future<RateLimitLease> RedisQueueingTokenBucketRateLimiter::AcquireAsyncCore(int p, const CancellationToken &ct) {
    check_limit(p, core_->options().TokenLimit);
    return core_->Submit(0, p, kQueueWait, ct);
}
void RedisQueueingTokenBucketRateLimiter::DisposeCore() { core_->Dispose(); }

// ------------------------------------------------------------------ approximate
RedisApproximateTokenBucketRateLimiter::RedisApproximateTokenBucketRateLimiter(
    const RedisApproximateTokenBucketRateLimiterOptions &o)
    : core_(std::make_unique<LimiterCore>(TBE_KIND_APPROXIMATE, o, false, "RedisApproximateTokenBucketRateLimiter")) {}
RedisApproximateTokenBucketRateLimiter::~RedisApproximateTokenBucketRateLimiter() = default;
std::optional<TimeSpan> RedisApproximateTokenBucketRateLimiter::IdleDuration() const { return core_->IdleDuration(); }
int RedisApproximateTokenBucketRateLimiter::GetAvailablePermits() {
    core_->ThrowIfDisposed();
    return core_->Run([this] { return core_->QueryApprox(0).available; });
}
bool RedisApproximateTokenBucketRateLimiter::TryReplenish() {
    if (core_->options().AutoReplenishment) return false;
    core_->ThrowIfDisposed();
    core_->Run([this] { core_->RefreshNow(); });
    return true;
}
std::string RedisApproximateTokenBucketRateLimiter::ToString() {
    const auto s = core_->Run([this] { return core_->QueryApprox(0); });
    char est[64];
    std::snprintf(est, sizeof est, "%.17g", s.est);
    for (int prec = 1; prec <= 17; ++prec) {  // shortest round-trip form, as .NET Core prints doubles
        char b[64];
        std::snprintf(b, sizeof b, "%.*g", prec, s.est);
        if (std::strtod(b, nullptr) == s.est) {
            std::snprintf(est, sizeof est, "%s", b);
            break;
        }
    }
    return "RedisApproximateTokenBucketRateLimiter Consumed: " +
           std::to_string((int32_t)((uint32_t)s.global + (uint32_t)s.local)) +
           " Available: " + std::to_string(s.available) + " Peer Count (Estimate): " + est;
}
RateLimitLease RedisApproximateTokenBucketRateLimiter::AttemptAcquireCore(int p) {
    check_limit(p, core_->options().TokenLimit);
    return core_->Submit(0, p, kApproxAttempt).get();
}
std::future<RateLimitLease> RedisApproximateTokenBucketRateLimiter::AcquireAsyncCore(int p, const CancellationToken &ct) {
    check_limit(p, core_->options().TokenLimit);
    core_->ThrowIfDisposed();  // A:124
    return core_->Submit(0, p, kApproxWait, ct);
}
void RedisApproximateTokenBucketRateLimiter::DisposeCore() { core_->Dispose(); }

// ------------------------------------------------------------------ registration
ServiceCollection &ServiceCollection::AddRedisTokenBucketRateLimiter(
    std::function<void(RedisTokenBucketRateLimiterOptions &)> configureOptions) {
    std::lock_guard<std::mutex> g(mu_);
    factory_ = [configureOptions] {
        RedisTokenBucketRateLimiterOptions o;
        configureOptions(o);
        return std::shared_ptr<RateLimiter>(std::make_shared<RedisTokenBucketRateLimiter>(o));
    };
    instance_.reset();
    return *this;
}

ServiceCollection &ServiceCollection::AddRedisApproximateTokenBucketRateLimiter(
    std::function<void(RedisApproximateTokenBucketRateLimiterOptions &)> configureOptions) {
    std::lock_guard<std::mutex> g(mu_);
    factory_ = [configureOptions] {
        RedisApproximateTokenBucketRateLimiterOptions o;
        configureOptions(o);
        return std::shared_ptr<RateLimiter>(std::make_shared<RedisApproximateTokenBucketRateLimiter>(o));
    };
    instance_.reset();
    return *this;
}

std::shared_ptr<RateLimiter> ServiceCollection::GetRequiredRateLimiter() {
    std::lock_guard<std::mutex> g(mu_);
    if (!instance_) {
        if (!factory_) throw std::logic_error("No service for type 'RateLimiter' has been registered.");
        instance_ = factory_();
    }
    return instance_;
}

}  // namespace tbe::rate_limiting
