// rate_limiting.hpp -- C++ host mirror of the reference's limiter API over the tbe C ABI.
//
// The reference (C#, net7.0) exposes System.Threading.RateLimiting limiters whose every
// decision is one StackExchange.Redis ScriptEvaluateAsync call (TB:63, PTB:42, A:439).
// There is no .NET toolchain in this image, so the host side above include/tbe.h is this
// C++ library: the same classes, option names, argument meaning and error behaviour,
// with the per-request script call replaced by a micro-batching submitter thread that
// turns concurrent callers into one batched engine call (arrival order = batch order,
// the order Redis would serialise the scripts in).  INTEGRATION.md shows the equivalent
// C# P/Invoke binding.
//
// Mapping (reference file:line -> here)
//   RedisTokenBucketRateLimiter            TokenBucket/RedisTokenBucketRateLimiter.cs:7-212
//   PartitionedRedisTokenBucketRateLimiter TokenBucket/PartitionedRedisTokenBucketRateLimiter.cs:7-212
//   RedisQueueingTokenBucketRateLimiter    TokenBucketWithQueue/RedisTokenBucketRateLimiter.cs:9-400
//   RedisApproximateTokenBucketRateLimiter ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs:9-599
//   *Options                               */Redis*Options.cs (TBO:9-85, QO, AO)
//   ServiceCollection::AddRedis*           ServiceCollectionExtensions.cs:10-26
// Method names follow the GA System.Threading.RateLimiting API (AttemptAcquire /
// AcquireAsync); the preview-5 names the reference overrides (AcquireCore /
// WaitAsyncCore) are the protected *Core virtuals.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "tbe.h"

namespace tbe::rate_limiting {

// ------------------------------------------------------------------ .NET value types
struct TimeSpan {  // System.TimeSpan: 100 ns ticks
    static constexpr int64_t TicksPerSecond = 10'000'000;
    int64_t ticks = 0;
    static TimeSpan FromTicks(int64_t t) { return TimeSpan{t}; }
    static TimeSpan FromSeconds(double s);
    static TimeSpan FromMilliseconds(double ms) { return FromSeconds(ms / 1000.0); }
    double TotalSeconds() const { return (double)ticks / (double)TicksPerSecond; }
    bool operator<(const TimeSpan &o) const { return ticks < o.ticks; }
    bool operator==(const TimeSpan &o) const { return ticks == o.ticks; }
};

// Exceptions with the .NET names the reference throws (TB:24-42, A:87-90, TB:158-164).
struct ArgumentException : std::invalid_argument {
    std::string ParamName;
    ArgumentException(const std::string &msg, std::string param)
        : std::invalid_argument(msg), ParamName(std::move(param)) {}
};
struct ArgumentNullException : ArgumentException {
    using ArgumentException::ArgumentException;
};
struct ArgumentOutOfRangeException : ArgumentException {
    using ArgumentException::ArgumentException;
};
struct ObjectDisposedException : std::logic_error {
    using std::logic_error::logic_error;
};
// An engine (device) error surfacing through a decision: the counterpart of a
// RedisException propagating out of ScriptEvaluateAsync (TB:63).
struct RateLimiterEngineException : std::runtime_error {
    tbe_status Status;
    RateLimiterEngineException(tbe_status st, const std::string &msg)
        : std::runtime_error(msg), Status(st) {}
};

// TaskCanceledException of a canceled queued wait (CancelQueueState.TrySetCanceled,
// Q:480-506, A:531-557).
struct OperationCanceledException : std::runtime_error {
    OperationCanceledException() : std::runtime_error("The operation was canceled.") {}
};

// System.Threading.CancellationToken / CancellationTokenSource, reduced to what the
// limiters use: CanBeCanceled, IsCancellationRequested and Register (callbacks run once,
// on the thread that calls Cancel, or at once when registered after it).
class CancellationToken {
public:
    CancellationToken() = default;  // CancellationToken.None
    bool CanBeCanceled() const { return (bool)s_; }
    bool IsCancellationRequested() const;
    // Returns a registration handle (0: nothing registered -- CancellationToken.None, or
    // already canceled, in which case fn has run).  Unregister(handle) removes a callback
    // that has not run (CancellationTokenRegistration.Dispose, Q:263, Q:303).
    uint64_t Register(std::function<void()> fn) const;
    void Unregister(uint64_t handle) const;
    size_t RegisteredCount() const;  // diagnostics (tests)
private:
    friend class CancellationTokenSource;
    struct State {
        std::mutex mu;
        bool canceled = false;
        uint64_t next = 1;
        std::map<uint64_t, std::function<void()>> callbacks;
    };
    explicit CancellationToken(std::shared_ptr<State> s) : s_(std::move(s)) {}
    std::shared_ptr<State> s_;
};

class CancellationTokenSource {
public:
    CancellationTokenSource() : s_(std::make_shared<CancellationToken::State>()) {}
    CancellationToken Token() const { return CancellationToken(s_); }
    bool IsCancellationRequested() const { return Token().IsCancellationRequested(); }
    void Cancel();
private:
    std::shared_ptr<CancellationToken::State> s_;
};

enum class QueueProcessingOrder { OldestFirst = 0, NewestFirst = 1 };

// RateLimitLease (the reference's private Lease classes, e.g. A:559-598).  Token-bucket
// leases hold nothing to give back, so a lease is a value.
class RateLimitLease {
public:
    explicit RateLimitLease(bool acquired, std::optional<TimeSpan> retry_after = std::nullopt)
        : acquired_(acquired), retry_after_(retry_after) {}
    bool IsAcquired() const { return acquired_; }
    std::vector<std::string> MetadataNames() const;                  // {"RETRY_AFTER"} (A:561)
    bool TryGetRetryAfter(TimeSpan &out) const;                      // MetadataName.RetryAfter
    std::string ToString() const;                                    // A:587-597
private:
    bool acquired_;
    std::optional<TimeSpan> retry_after_;
};

// The role of Redis TIME (TB:202): microseconds since the Unix epoch.  Injectable so
// tests can drive the limiters deterministically.
using Clock = std::function<int64_t()>;
int64_t SystemClockMicros();

// Diagnostic hook: every engine call the submitter makes, with its inputs and replies
// (status: 0/1 granted for the token bucket, TBE_WAIT_* otherwise).
struct BatchTrace {
    int mode;  // BatchMode
    uint64_t n;
    const uint64_t *keys;
    const int32_t *permits;
    const int64_t *ts_us;
    const uint8_t *status;
    const int32_t *remaining;
};
enum BatchMode { kTbAcquire = 0, kQueueWait = 1, kQueueAttempt = 2, kApproxWait = 3, kApproxAttempt = 4 };

// ------------------------------------------------------------------ options
// RedisTokenBucketRateLimiterOptions (TBO:9-85).  The Redis connection settings
// (Configuration, ConfigurationOptions, ConnectionMultiplexerFactory, ProfilingSession)
// become the engine settings below: the "connection" is a GPU.
struct RedisTokenBucketRateLimiterOptions {
    TimeSpan ReplenishmentPeriod = TimeSpan::FromSeconds(1);      // TBO:14-22
    int TokensPerPeriod = 0;                                      // TBO:24-32
    int TokenLimit = 0;                                           // TBO:43
    std::string InstanceName;                                     // TBO:65 (key prefix)
    int Device = -1;               // HIP device ordinal (-1: current)
    uint64_t PartitionLimit = 1u << 20;  // partitioned limiters: distinct resource ids
    uint64_t MaxBatch = 1u << 16;  // largest micro-batch one engine call takes
    Clock TimeSource;              // default SystemClockMicros
    std::function<void(const BatchTrace &)> OnBatch;  // diagnostics (tests)
    double FillRatePerSecond() const;                             // TBO:82-85
};

// RedisQueueingTokenBucketRateLimiterOptions (TokenBucketWithQueue/...Options.cs).
struct RedisQueueingTokenBucketRateLimiterOptions : RedisTokenBucketRateLimiterOptions {
    int QueueLimit = 0;
    ::tbe::rate_limiting::QueueProcessingOrder QueueProcessingOrder =
        ::tbe::rate_limiting::QueueProcessingOrder::OldestFirst;
    // Timer-driven replenishment every ReplenishmentPeriod (the reference's timer);
    // false: call TryReplenish() yourself (as System.Threading.RateLimiting allows).
    bool AutoReplenishment = true;
    // Approximate limiter only: queue entries per key kept for zero-permit waits, which
    // the reference queues without bound while throttled (A:127-181; include/tbe.h).
    int ZeroWaitSlots = 4;
};

// RedisApproximateTokenBucketRateLimiterOptions (ApproximateTokenBucket/...Options.cs).
struct RedisApproximateTokenBucketRateLimiterOptions : RedisQueueingTokenBucketRateLimiterOptions {};

// ------------------------------------------------------------------ base classes
class RateLimiter {  // System.Threading.RateLimiting.RateLimiter
public:
    virtual ~RateLimiter() = default;
    virtual std::optional<TimeSpan> IdleDuration() const = 0;
    virtual int GetAvailablePermits() = 0;
    // Base-class argument validation: permitCount < 0 -> ArgumentOutOfRangeException.
    RateLimitLease AttemptAcquire(int permitCount = 1);
    // A queued request whose token is canceled completes with OperationCanceledException
    // (A:166-175); a request decided at once ignores the token, as in the reference.
    std::future<RateLimitLease> AcquireAsync(int permitCount = 1, CancellationToken ct = {});
    void Dispose() { DisposeCore(); }
protected:
    virtual RateLimitLease AttemptAcquireCore(int permitCount) = 0;
    virtual std::future<RateLimitLease> AcquireAsyncCore(int permitCount, const CancellationToken &ct) = 0;
    virtual void DisposeCore() = 0;
};

template <class TResource>
class PartitionedRateLimiter {  // System.Threading.RateLimiting.PartitionedRateLimiter<T>
public:
    virtual ~PartitionedRateLimiter() = default;
    virtual int GetAvailablePermits(const TResource &resource) = 0;
    RateLimitLease AttemptAcquire(const TResource &resource, int permitCount = 1) {
        if (permitCount < 0) throw ArgumentOutOfRangeException("permitCount must be >= 0", "permitCount");
        return AttemptAcquireCore(resource, permitCount);
    }
    std::future<RateLimitLease> AcquireAsync(const TResource &resource, int permitCount = 1,
                                             CancellationToken ct = {}) {
        if (permitCount < 0) throw ArgumentOutOfRangeException("permitCount must be >= 0", "permitCount");
        return AcquireAsyncCore(resource, permitCount, ct);
    }
    void Dispose() { DisposeCore(); }
protected:
    virtual RateLimitLease AttemptAcquireCore(const TResource &resource, int permitCount) = 0;
    virtual std::future<RateLimitLease> AcquireAsyncCore(const TResource &resource, int permitCount,
                                                         const CancellationToken &ct) = 0;
    virtual void DisposeCore() = 0;
};

namespace detail {
class LimiterCore;  // engine + key directory + submitter thread (rate_limiting.cpp)
}

// ------------------------------------------------------------------ token bucket
// TB:7-212.  One bucket (BucketId = InstanceName).  AttemptAcquire runs the real decision
// (the reference's AcquireCore is a stub returning FailedLease, TB:53-56).
class RedisTokenBucketRateLimiter final : public RateLimiter {
public:
    explicit RedisTokenBucketRateLimiter(const RedisTokenBucketRateLimiterOptions &options);
    ~RedisTokenBucketRateLimiter() override;
    std::optional<TimeSpan> IdleDuration() const override { return std::nullopt; }  // TB:20
    int GetAvailablePermits() override;                                               // TB:48-51
protected:
    RateLimitLease AttemptAcquireCore(int permitCount) override;
    std::future<RateLimitLease> AcquireAsyncCore(int permitCount, const CancellationToken &ct) override;          // TB:58-82
    void DisposeCore() override;                                                      // TB:85-109
private:
    std::unique_ptr<detail::LimiterCore> core_;
};

// PTB:7-212.  BucketId = InstanceName + resourceID (PTB:42), mapped to a dense key.
// GetAvailablePermits(resourceID) reports the last script reply for that bucket (the
// reference returns 0, PTB:25-28).
class PartitionedRedisTokenBucketRateLimiter final : public PartitionedRateLimiter<std::string> {
public:
    explicit PartitionedRedisTokenBucketRateLimiter(const RedisTokenBucketRateLimiterOptions &options);
    ~PartitionedRedisTokenBucketRateLimiter() override;
    int GetAvailablePermits(const std::string &resourceID) override;
    // Frees the keys of buckets Redis would have expired (TB:232-235) for new resource
    // ids; runs by itself when all PartitionLimit keys are taken.  Returns the number freed.
    uint64_t ReclaimExpired();
protected:
    RateLimitLease AttemptAcquireCore(const std::string &resourceID, int permitCount) override;
    std::future<RateLimitLease> AcquireAsyncCore(const std::string &resourceID, int permitCount,
                                                 const CancellationToken &ct) override;
    void DisposeCore() override;
private:
    std::unique_ptr<detail::LimiterCore> core_;
};

// ------------------------------------------------------------------ token bucket with queue
// Q:9-400 (commented out upstream; semantics fixed in DESIGN.md §2b).  WaitAsync leases,
// else queues (QueueLimit, QueueProcessingOrder), and queued requests complete at the
// replenish ticks.
class RedisQueueingTokenBucketRateLimiter final : public RateLimiter {
public:
    explicit RedisQueueingTokenBucketRateLimiter(const RedisQueueingTokenBucketRateLimiterOptions &options);
    ~RedisQueueingTokenBucketRateLimiter() override;
    std::optional<TimeSpan> IdleDuration() const override { return std::nullopt; }  // Q:29
    int GetAvailablePermits() override;                                               // Q:57-60
    bool TryReplenish();  // one replenish tick now; false when AutoReplenishment is on
protected:
    RateLimitLease AttemptAcquireCore(int permitCount) override;
    std::future<RateLimitLease> AcquireAsyncCore(int permitCount, const CancellationToken &ct) override;          // Q:67-134
    void DisposeCore() override;
private:
    std::unique_ptr<detail::LimiterCore> core_;
};

// ------------------------------------------------------------------ approximate
// A:9-599.  Local tier per instance, periodically synced with the global tier.  This
// limiter is the only client of its engine's global-tier replica; multi-client (multi-GPU)
// sync goes through the cluster layer (cluster.py approx_epoch over RCCL).
class RedisApproximateTokenBucketRateLimiter final : public RateLimiter {
public:
    explicit RedisApproximateTokenBucketRateLimiter(const RedisApproximateTokenBucketRateLimiterOptions &options);
    ~RedisApproximateTokenBucketRateLimiter() override;
    std::optional<TimeSpan> IdleDuration() const override;                            // A:34
    int GetAvailablePermits() override;                                               // A:81
    bool TryReplenish();  // one RefreshAsync (A:412-508) now; false when AutoReplenishment is on
    std::string ToString();                                                           // A:510-513
protected:
    RateLimitLease AttemptAcquireCore(int permitCount) override;                     // A:84-113
    std::future<RateLimitLease> AcquireAsyncCore(int permitCount, const CancellationToken &ct) override;          // A:116-183
    void DisposeCore() override;                                                      // A:274-300
private:
    std::unique_ptr<detail::LimiterCore> core_;
};

// ------------------------------------------------------------------ registration
// ServiceCollectionExtensions (SCE:10-26): registers a singleton RateLimiter built from
// configured options.  Resolution constructs it on first use (as the DI container does).
class ServiceCollection {
public:
    ServiceCollection &AddRedisTokenBucketRateLimiter(
        std::function<void(RedisTokenBucketRateLimiterOptions &)> configureOptions);
    ServiceCollection &AddRedisApproximateTokenBucketRateLimiter(
        std::function<void(RedisApproximateTokenBucketRateLimiterOptions &)> configureOptions);
    // GetRequiredService<RateLimiter>(): the last registration wins (MS.DI semantics).
    std::shared_ptr<RateLimiter> GetRequiredRateLimiter();
private:
    std::mutex mu_;
    std::function<std::shared_ptr<RateLimiter>()> factory_;
    std::shared_ptr<RateLimiter> instance_;
};

}  // namespace tbe::rate_limiting
