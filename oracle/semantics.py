"""CPU restatement of the reference's rate-limiting decision semantics.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker (or, for bench, as the timed CPU baseline) -- never as the product path.
The product path is the HIP engine behind ``include/tbe.h``; it fails loudly when
its shared library is missing and never falls back to this code.

Parity status: the reference (C# + Lua run inside Redis) has no tests, fixtures or
golden vectors, and neither .NET, Redis nor a Lua VM exists in this
image.  This restatement is pinned by
  (1) the hand-derived known-answer tests of SURVEY.md Appendix A.6,
  (2) bit-for-bit agreement with the independent C restatement ``oracle/tb_ref.c``,
  (3) golden vectors produced by executing the reference's own Lua script text
      (read from /root/reference at fixture-generation time) in the in-repo Lua
      subset interpreter ``oracle/lua_replay.py`` (tests/golden/make_golden.py).
Redis/SE.Redis/.NET conversion behaviour is restated from their published
semantics; it is not pinned by any artefact the
reference ships.

Every arithmetic step is IEEE-754 binary64 round-to-nearest with no FMA -- Python
floats give exactly that.  Argument order of ``math.min``/``math.max`` follows Lua
5.1's ``lmathlib.c`` (first argument kept unless a later one is strictly
better), which fixes signed-zero/NaN behaviour.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

US_PER_S = 1_000_000
TICKS_PER_SECOND = 10_000_000          # System.TimeSpan.TicksPerSecond
TTL_MAX_S = 31_536_000                  # TB:234 upper clamp (1 year)
APPROX_TTL_S = 86_400                   # A:268


# ---------------------------------------------------------------- Lua / Redis / .NET helpers
def lua_max(a: float, b: float) -> float:
    """Lua 5.1 ``math.max(a, b)``: keeps ``a`` unless ``b > a``."""
    return b if b > a else a


def lua_min(a: float, b: float) -> float:
    """Lua 5.1 ``math.min(a, b)``: keeps ``a`` unless ``b < a``."""
    return b if b < a else a


def new_t_of(ts_us: int) -> float:
    """``now[1] + (now[2] / 1000000)`` over Redis ``TIME`` (TB:202-203, A:241-242).

    ``TIME`` returns two integer strings (seconds, microseconds); Lua coerces
    them to numbers, divides the microseconds by 1e6 (one correctly rounded
    division) and adds (one rounding).  The build injects ``ts_us`` (>= 0)."""
    sec, usec = divmod(ts_us, US_PER_S)
    return float(sec) + (float(usec) / 1000000.0)


def fill_rate_per_second(tokens_per_period: int, period_ticks: int) -> float:
    """``FillRatePerSecond = _tokensPerPeriod / _replenishmentPeriod.TotalSeconds``
    (TBO:82-85, AO:97-100); .NET 7 ``TimeSpan.TotalSeconds`` = ticks / 1e7."""
    total_seconds = float(period_ticks) / float(TICKS_PER_SECOND)
    if total_seconds == 0.0:
        return math.inf
    return float(tokens_per_period) / total_seconds


def tb_ttl_seconds(capacity: int, fill_rate: float) -> int:
    """``math.ceil(math.min(math.max(capacity / fill_rate, 1), 31536000))`` (TB:234)."""
    return int(math.ceil(lua_min(lua_max(float(capacity) / fill_rate, 1.0), float(TTL_MAX_S))))


def redis_int_reply(x: float) -> int:
    """Lua number -> RESP integer: C cast to ``long long`` (truncation toward 0)."""
    return int(x)


def lua_tostring(x: float) -> str:
    """Lua 5.1 ``tostring(number)`` = ``LUA_NUMBER_FMT`` "%.14g" (A:270)."""
    return "%.14g" % x


def dotnet_round_half_even(x: float) -> float:
    """``Math.Round(double)`` (banker's rounding, A:443)."""
    if math.isinf(x) or math.isnan(x):
        return x
    return float(round(x))  # Python's round() on floats is round-half-even


class ArgumentOutOfRange(ValueError):
    """Mirrors ArgumentOutOfRangeException (permitCount < 0, or > TokenLimit in A/Q)."""


# ---------------------------------------------------------------- token-bucket acquire script
@dataclass
class TokenBucketConfig:
    """Inputs of ``GetAcquireLuaScript(capacity, fillRate)`` (TB:176-185)."""

    token_limit: int                 # TBO:43 -> Lua ``capacity`` (TB:184)
    fill_rate: float                 # TBO:80 -> Lua ``fill_rate`` (TB:185), raw f64 bits

    @staticmethod
    def from_options(token_limit: int, tokens_per_period: int, period_ticks: int) -> "TokenBucketConfig":
        # Constructor validation, TB:29-37.
        if token_limit <= 0 or tokens_per_period <= 0:
            raise ValueError("Both TokenLimit and TokensPerPeriod must be set to values greater than 0.")
        if period_ticks < 0:
            raise ValueError("ReplenishmentPeriod must be set to a value greater than or equal to TimeSpan.Zero.")
        rate = fill_rate_per_second(tokens_per_period, period_ticks)
        if not math.isfinite(rate):
            # ReplenishmentPeriod == 0 passes TB:34 but interpolates "∞" into the
            # script, which Redis rejects at compile time.
            raise ValueError("ReplenishmentPeriod must be > 0 (fill rate would be infinite)")
        return TokenBucketConfig(token_limit, rate)


@dataclass
class BucketState:
    v: float        # Redis hash field ``v`` (tokens), stored with round-trip precision
    t_us: int       # injected TIME of the last grant; field ``t`` = new_t_of(t_us)


class TokenBucketTable:
    """The Redis key space seen by the acquire script (TB:181-238), one hash per key.

    A key is *present* from its first grant until its TTL (TB:232-235) lapses with no
    further grant.  Redis' passive expiry compares the command-time snapshot in ms
    (frozen for the duration of a script) with ``grant_ms + ttl_s * 1000``; the build
    models both snapshots as ``ts_us // 1000``."""

    def __init__(self, cfg: TokenBucketConfig):
        self.cfg = cfg
        self.cap = float(cfg.token_limit)
        self.rate = cfg.fill_rate
        self.ttl_ms = tb_ttl_seconds(cfg.token_limit, cfg.fill_rate) * 1000
        self.state: Dict[int, BucketState] = {}

    # HGETALL with passive expiry (TB:210-215)
    def load(self, key: int, ts_us: int) -> Optional[BucketState]:
        st = self.state.get(key)
        if st is None:
            return None
        if ts_us // 1000 > st.t_us // 1000 + self.ttl_ms:
            del self.state[key]
            return None
        return st

    def refill(self, key: int, ts_us: int) -> Tuple[float, float, Optional[BucketState]]:
        """TB:202-221: returns (new_t, x, prev) where x is the refilled, clamped count."""
        new_t = new_t_of(ts_us)                                   # TB:202-203
        prev = self.load(key, ts_us)                              # TB:210
        if prev is None:                                          # TB:213-215
            pv, pt = self.cap, new_t
        else:                                                     # TB:211-212
            pv, pt = prev.v, new_t_of(prev.t_us)
        delta_t = lua_max(0.0, new_t - pt)                        # TB:218
        x = lua_max(0.0, lua_min(self.cap, pv + (delta_t * self.rate)))   # TB:221
        return new_t, x, prev

    def acquire(self, key: int, permits: int, ts_us: int) -> Tuple[bool, int]:
        """One ``ScriptEvaluateAsync(_acquireScript, {BucketId, PermitCount})`` (TB:63)
        plus the C# reply parse (TB:64-81).  Returns (granted, remaining)."""
        if permits < 0:
            raise ArgumentOutOfRange("permitCount")
        _, x, _ = self.refill(key, ts_us)
        success = x >= float(permits)                             # TB:224
        if success:
            x = x - float(permits)                                # TB:227
            self.state[key] = BucketState(x, ts_us)               # TB:230 HSET v,t (+ EXPIRE TB:234-235)
        # TB:238 ``return {success, new_v}``: true -> 1, false -> nil (-> 0 in SE.Redis),
        # new_v -> RESP integer (truncation).  TB:71-81 reads them back.
        return success, redis_int_reply(x)

    def acquire_batch(self, keys, permits, ts_us) -> Tuple[List[int], List[int]]:
        granted, remaining = [], []
        for k, p, t in zip(keys, permits, ts_us):
            g, r = self.acquire(int(k), int(p), int(t))
            granted.append(1 if g else 0)
            remaining.append(r)
        return granted, remaining

    def query(self, key: int, ts_us: Optional[int] = None) -> Optional[Tuple[float, float]]:
        """(v, t) exactly as stored in the Redis hash, or None when absent/expired."""
        st = self.state.get(key) if ts_us is None else self.load(key, ts_us)
        if st is None:
            return None
        return st.v, new_t_of(st.t_us)


# ---------------------------------------------------------------- approximate: global sync script
@dataclass
class ApproxGlobalState:
    v: float      # decayed consumed count (A:258)
    p: float      # EWMA of the gap between sync calls (A:262)
    t_us: int     # injected TIME of the last sync; field t = new_t_of(t_us)


class ApproxGlobalTable:
    """The Redis key space seen by the approximate limiter's sync script (A:221-270)."""

    def __init__(self, decay_rate: float):
        self.rate = decay_rate
        self.ttl_ms = APPROX_TTL_S * 1000
        self.state: Dict[str, ApproxGlobalState] = {}

    def load(self, bucket: str, ts_us: int) -> Optional[ApproxGlobalState]:
        st = self.state.get(bucket)
        if st is not None and ts_us // 1000 > st.t_us // 1000 + self.ttl_ms:  # EXPIRE 86400 (A:268)
            del self.state[bucket]
            return None
        return st

    def sync(self, bucket: str, local_count: int, ts_us: int) -> Tuple[int, float, str]:
        """One ``ScriptEvaluateAsync(_syncScript, {BucketId, LocalCount})`` (A:439) and the
        reply parse (A:440-442): returns (global score, period, period string)."""
        new_t = new_t_of(ts_us)                                          # A:241-242
        prev = self.load(bucket, ts_us)                                  # A:245
        if prev is None:                                                 # A:250-252
            pv, pp, pt = 0.0, 0.0, new_t
        else:                                                            # A:247-249
            pv, pp, pt = prev.v, prev.p, new_t_of(prev.t_us)
        count = float(local_count)                                       # A:223 tonumber
        delta_t = lua_max(0.0, new_t - pt)                               # A:255
        new_v = lua_max(0.0, pv - (delta_t * self.rate)) + count        # A:258
        new_p = (pp * 0.8) + (delta_t * 0.2)                             # A:262
        self.state[bucket] = ApproxGlobalState(new_v, new_p, ts_us)      # A:265 (+ EXPIRE A:268)
        period_str = lua_tostring(new_p)                                 # A:270 tostring(new_p)
        return redis_int_reply(new_v), float(period_str), period_str


def instance_count_estimate(replenishment_seconds: float, period: float) -> float:
    """``Math.Max(1, Math.Round(ReplenishmentPeriod.TotalSeconds / period))`` (A:443);
    period 0 gives +inf (double division), Max(1, inf) = inf."""
    if period == 0.0:
        q = math.inf if replenishment_seconds > 0 else math.nan
    else:
        q = replenishment_seconds / period
    r = dotnet_round_half_even(q)
    if math.isnan(r):
        return math.nan  # Math.Max(1, NaN) = NaN in .NET
    return max(1.0, r)


# ---------------------------------------------------------------- token bucket with queue
# TokenBucketWithQueue/RedisTokenBucketRateLimiter.cs ("Q") is commented out and does not
# compile (it uses members it never declares), so its semantics are
# fixed here by composing its control flow with the TB acquire script as the only
# token source:
#   WaitAsyncCore           Q:67-134   admission (lease, else queue, else fail)
#   TryLeaseUnsynchronized  Q:136-165  OldestFirst never leases past a non-empty queue
#   RefreshAsync drain      Q:237-271  head (OldestFirst) / tail (NewestFirst) while granted
#   Deque order             DQ:19-94   EnqueueTail, DequeueHead, PeekTail/DequeueTail
# Decisions on undefined behaviour: a lease IS one TB script call
# (`AvailableTokens >= count` + consume is the script's x >= p + HSET); p == 0 goes
# straight through the script (never queued: unbounded zero-permit queueing is a
# reference quirk); p > TokenLimit is rejected per request
# (ArgumentOutOfRangeException, Q:70-73).

OLDEST_FIRST, NEWEST_FIRST = 0, 1
ST_FAILED, ST_GRANTED, ST_QUEUED, ST_REJECTED = 0, 1, 2, 3
REMAINING_NOT_EVALUATED = -1   # the script was not called for this request


@dataclass
class QueueEntry:
    request_id: int
    permits: int


class QueueingTokenBucketTable:
    """Per-key bucket (TB script) + per-key deque of waiting requests."""

    def __init__(self, cfg: TokenBucketConfig, queue_limit: int, order: int):
        if queue_limit < 0:
            raise ValueError("QueueLimit must be set to a value greater than or equal to 0.")
        self.tb = TokenBucketTable(cfg)
        self.queue_limit = queue_limit
        self.order = order
        self.queues: Dict[int, List[QueueEntry]] = {}
        self.qsum: Dict[int, int] = {}

    def acquire(self, key: int, permits: int, ts_us: int, request_id: int):
        """Returns (status, remaining, evicted_ids)."""
        if permits < 0:
            raise ArgumentOutOfRange("permitCount")
        if permits > self.tb.cfg.token_limit:                       # Q:70-73
            return ST_REJECTED, REMAINING_NOT_EVALUATED, []
        q = self.queues.setdefault(key, [])
        qsum = self.qsum.get(key, 0)
        remaining = REMAINING_NOT_EVALUATED
        if permits == 0 or not (q and self.order == OLDEST_FIRST):  # Q:153
            granted, remaining = self.tb.acquire(key, permits, ts_us)
            if granted:
                return ST_GRANTED, remaining, []
        evicted = []
        if self.queue_limit - qsum < permits:                        # Q:92
            if self.order == NEWEST_FIRST and permits <= self.queue_limit:   # Q:94-109
                while self.queue_limit - qsum < permits:
                    e = q.pop(0)                                     # DequeueHead
                    qsum -= e.permits
                    evicted.append(e.request_id)
            else:
                self.qsum[key] = qsum
                return ST_FAILED, remaining, []                      # Q:113
        q.append(QueueEntry(request_id, permits))                    # Q:128 EnqueueTail
        self.qsum[key] = qsum + permits
        return ST_QUEUED, remaining, evicted

    def attempt(self, key: int, permits: int, ts_us: int):
        """AttemptAcquire: TryLeaseUnsynchronized only (Q:136-165), never queues.
        Returns (status, remaining)."""
        if permits < 0:
            raise ArgumentOutOfRange("permitCount")
        if permits > self.tb.cfg.token_limit:
            return ST_REJECTED, REMAINING_NOT_EVALUATED
        if permits == 0 or not (self.queues.get(key) and self.order == OLDEST_FIRST):
            granted, remaining = self.tb.acquire(key, permits, ts_us)
            return (ST_GRANTED if granted else ST_FAILED), remaining
        return ST_FAILED, REMAINING_NOT_EVALUATED

    def refresh(self, ts_us: int):
        """Drain every non-empty queue at one replenish tick (Q:237-271).  Returns the
        grant log [(key, request_id, remaining)] in (key, drain order)."""
        log = []
        for key in sorted(self.queues):
            q = self.queues[key]
            while q:
                e = q[0] if self.order == OLDEST_FIRST else q[-1]    # PeekHead / PeekTail
                granted, remaining = self.tb.acquire(key, e.permits, ts_us)
                if not granted:
                    break
                if self.order == OLDEST_FIRST:
                    q.pop(0)                                          # DequeueHead
                else:
                    q.pop()                                           # DequeueTail
                self.qsum[key] -= e.permits
                log.append((key, e.request_id, remaining))
        return log

    def queue_of(self, key: int) -> List[Tuple[int, int]]:
        return [(e.request_id, e.permits) for e in self.queues.get(key, [])]

    def cancel(self, key: int, request_id: int) -> bool:
        """CancelQueueState.TrySetCanceled (Q:480-506): True iff the request was queued on
        `key`; _queueCount -= its permits (Q:499).  Build decision: the
        registration leaves the deque at once instead of waiting for the drain (Q:256-262),
        so it neither consumes tokens nor holds up the entries behind it."""
        q = self.queues.get(key, [])
        for j, e in enumerate(q):
            if e.request_id == request_id:
                del q[j]
                self.qsum[key] -= e.permits
                return True
        return False


# ---------------------------------------------------------------- approximate: local tier
# ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs ("A") as one client's
# local tier per key (partitioned: BucketId = InstanceName + key, cf. PTB:42):
#   AvailableTokens        A:37     max(0, (int)ceil((TokenLimit - global) / est) - local)
#   AcquireCore            A:84-113 (sync: never queues)
#   WaitAsyncCore          A:116-183 (async: may queue)
#   TryLeaseUnsynchronized A:185-214
#   RefreshAsync           A:412-508 (swap local -> count, sync script, drain)
# Zero-permit WaitAsync while throttled (A:127-181): TryLease fails (availableTokens != 0)
# and `QueueLimit - _queueCount < 0` never holds, so the registration queues with Count 0,
# holds no queue permits and completes at the first drain that reaches it (A:474:
# AvailableTokens >= 0).  The reference queues any number of them;
# the build gives each key `zero_slots` of them, beyond which the wait FAILS.
AP_FAILED, AP_GRANTED, AP_QUEUED, AP_REJECTED = 0, 1, 2, 3
INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def wrap32(x: int) -> int:
    """C# unchecked int32 arithmetic."""
    return ((x + 2 ** 31) % 2 ** 32) - 2 ** 31


def dotnet_double_to_int(x: float) -> int:
    """C# ``(int)double`` (unchecked; .NET 7 on x64 saturates NaN/overflow to INT32_MIN,
    the cvttsd2si result; in-range values truncate toward zero)."""
    if math.isnan(x) or x >= 2147483648.0 or x <= -2147483649.0:
        return INT32_MIN
    return int(x)


@dataclass
class ApproxLocal:
    local: int = 0            # _localThrottleScore
    global_: int = 0          # _globalThrottleScore
    est: float = 1.0          # _instanceCountEstimate
    queue: List[QueueEntry] = field(default_factory=list)
    qcount: int = 0           # _queueCount


class ApproxClient:
    """One client process's local tier for every key (A:9-599)."""

    def __init__(self, token_limit: int, tokens_per_period: int, period_ticks: int,
                 queue_limit: int, order: int, zero_slots: int = 4):
        if token_limit <= 0 or tokens_per_period <= 0:
            raise ValueError("Both TokenLimit and TokensPerPeriod must be set to values greater than 0.")
        if queue_limit < 0:
            raise ValueError("QueueLimit must be set to a value greater than or equal to 0.")
        if period_ticks < 0:
            raise ValueError("ReplenishmentPeriod must be >= 0")
        self.token_limit = token_limit
        self.queue_limit = queue_limit
        self.order = order
        self.zero_slots = zero_slots
        self.period_seconds = float(period_ticks) / float(TICKS_PER_SECOND)
        self.decay_rate = fill_rate_per_second(tokens_per_period, period_ticks)
        self.keys: Dict[int, ApproxLocal] = {}

    def st(self, key: int) -> ApproxLocal:
        s = self.keys.get(key)
        if s is None:
            s = self.keys[key] = ApproxLocal()
        return s

    def cap_of(self, s: ApproxLocal) -> int:
        """(int)Math.Ceiling((TokenLimit - global) / est)  (A:37; int / double division)."""
        q = float(wrap32(self.token_limit - s.global_)) / s.est
        return dotnet_double_to_int(float(math.ceil(q)) if math.isfinite(q) else q)

    def available(self, s: ApproxLocal) -> int:
        """A:37: Math.Max(0, cap - _localThrottleScore) with unchecked int arithmetic."""
        return max(0, wrap32(self.cap_of(s) - s.local))

    def try_lease(self, s: ApproxLocal, p: int) -> bool:
        """A:185-214 (returns True on lease)."""
        avail = self.available(s)
        if avail >= p and avail != 0:
            if p == 0:
                return True
            if s.qcount == 0 or self.order == NEWEST_FIRST:
                s.local = wrap32(s.local + p)
                return True
        return False

    def acquire(self, key: int, p: int) -> int:
        """AcquireCore (A:84-113)."""
        if p < 0:
            raise ArgumentOutOfRange("permitCount")
        if p > self.token_limit:
            return AP_REJECTED
        s = self.st(key)
        if p == 0:
            return AP_GRANTED if self.available(s) > 0 else AP_FAILED
        return AP_GRANTED if self.try_lease(s, p) else AP_FAILED

    def wait(self, key: int, p: int, request_id: int):
        """WaitAsyncCore (A:116-183): (status, evicted ids)."""
        if p < 0:
            raise ArgumentOutOfRange("permitCount")
        if p > self.token_limit:
            return AP_REJECTED, []
        s = self.st(key)
        if p == 0 and self.available(s) > 0:
            return AP_GRANTED, []
        if self.try_lease(s, p):
            return AP_GRANTED, []
        if p == 0:
            # queued with Count 0 (A:141 never fails for 0); bounded by zero_slots per key
            if sum(1 for e in s.queue if e.permits == 0) >= self.zero_slots:
                return AP_FAILED, []
            s.queue.append(QueueEntry(request_id, 0))
            return AP_QUEUED, []
        evicted = []
        if self.queue_limit - s.qcount < p:
            if self.order == NEWEST_FIRST and p <= self.queue_limit:
                while self.queue_limit - s.qcount < p:
                    e = s.queue.pop(0)
                    s.qcount -= e.permits
                    evicted.append(e.request_id)
            else:
                return AP_FAILED, []
        s.queue.append(QueueEntry(request_id, p))
        s.qcount += p
        return AP_QUEUED, evicted

    def cancel(self, key: int, request_id: int) -> bool:
        """CancelQueueState.TrySetCanceled (A:545-556): True iff the request was queued on
        `key`; _queueCount -= its permits.  Removed at once, so the drain
        never reaches it and the A:489 double add-back cannot happen."""
        s = self.keys.get(key)
        if s is None:
            return False
        for j, e in enumerate(s.queue):
            if e.request_id == request_id:
                del s.queue[j]
                s.qcount -= e.permits
                return True
        return False

    def collect(self) -> Dict[int, int]:
        """A:430-435: swap every key's local score to 0; returns the counts."""
        out = {}
        for k, s in self.keys.items():
            out[k] = s.local
            s.local = 0
        return out

    def apply_sync(self, key: int, global_score: int, period: float):
        """A:441-443"""
        s = self.st(key)
        s.global_ = global_score
        s.est = instance_count_estimate(self.period_seconds, period)

    def drain(self):
        """A:462-501 over every key (in key order): [(key, request_id)] granted."""
        log = []
        for k in sorted(self.keys):
            s = self.keys[k]
            while s.queue:
                e = s.queue[0] if self.order == OLDEST_FIRST else s.queue[-1]
                if self.available(s) >= e.permits:
                    if self.order == OLDEST_FIRST:
                        s.queue.pop(0)
                    else:
                        s.queue.pop()
                    s.qcount -= e.permits
                    s.local = wrap32(s.local + e.permits)
                    log.append((k, e.request_id))
                else:
                    break
        return log


def approx_refresh_all(clients: List[ApproxClient], table: ApproxGlobalTable, ts_us: int,
                       stagger_us: int, keys):
    """One refresh epoch of N clients sharing one global tier: client r syncs at
    ts_us + r*stagger_us, in client order (the sequential Redis script calls of SURVEY.md
    §8e option 2), then drains its queues.  `keys` are the keys synced this epoch
    (in the reference every limiter instance syncs every period)."""
    counts = [c.collect() for c in clients]
    logs = []
    for r, c in enumerate(clients):
        for k in keys:
            g, period, _ = table.sync(f"approx:{k}", counts[r].get(k, 0), ts_us + r * stagger_us)
            c.apply_sync(k, g, period)
        logs.append(c.drain())
    return logs
