// Cross-process service state in POSIX shared memory: the response cache (TTL + LRU, cachetools
// TTLCache semantics) and the fixed-window rate-limit counters (slowapi/limits memory storage
// semantics), shared by every API worker process of one service (SURVEY.md §6 "HTTP tier",
// §7.3 hard part 6).  The reference keeps both process-local (`/root/reference/app.py:125,128`)
// because it runs one uvicorn worker (`app.py:400`); with N workers behind one port a miss
// answered by worker A must be `from_cache: true` on worker B (`app.py:312-322`) and a client's
// 10/minute must be counted once, not N times.
//
// Layout (one mmap'd segment, fixed size, no pointers — only indices — so every process can map
// it at a different address):
//   Header | cache hash buckets (int32) | cache entries | limiter slots
// Keys are 128-bit digests computed by the caller (BLAKE2b-128 of the key text, Python side), so
// arbitrarily long queries cost a fixed 16 bytes; values (generated commands) are stored inline up
// to `value_max` bytes (a longer value is not stored: the caller serves it uncached).
// A robust process-shared mutex guards everything: a worker that dies holding it leaves the
// segment consistent (every mutation is completed before unlock, and EOWNERDEAD marks the
// mutex consistent again).  Times are passed in by the caller (its injectable timer):
// CLOCK_MONOTONIC / wall clock are system-wide, so all workers agree.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace ka {

class SharedState {
 public:
  static constexpr uint64_t kMagic = 0x4b41535354415445ull;   // "KASSTATE"
  static constexpr uint32_t kVersion = 3;
  // DP routing load table: in-flight requests per (API worker, engine replica).  Each worker writes
  // only its own row (single writer, lock-free); a router picks the replica with the least total
  // over all rows, so W workers balance N replicas as one router would.
  static constexpr uint32_t kMaxWorkers = 64, kMaxReplicas = 64;

  struct Header {
    uint64_t magic;
    uint32_t version, cache_cap, value_max, nbuckets, lim_cap, pad0;
    uint64_t entry_bytes, total_bytes;
    pthread_mutex_t mu;
    int32_t lru_head, lru_tail, free_head;   // LRU: head = least recently used
    uint32_t count;
    uint64_t hits, misses, sets, evictions, lim_used;
    uint64_t owner_deaths;   // lock holders that died (each reset the segment)
    int64_t load[kMaxWorkers][kMaxReplicas];   // not covered by the mutex, not cleared by a reset
  };
  struct Entry {
    uint64_t k0, k1;
    double expires;
    int32_t prev, next, hnext;
    uint32_t vlen;
    // char value[value_max] follows
  };
  struct Slot {   // limiter: open addressing, linear probing
    uint64_t k0, k1;
    double window_end;
    uint32_t count, state;   // state: 0 empty, 1 used
  };

  // Create (exclusive) or attach to the named segment.  `create` with an existing name attaches.
  static SharedState open(const std::string& name, uint32_t cache_cap, uint32_t value_max, uint32_t lim_cap) {
    SharedState s;
    s.name_ = name;
    int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    bool creator = fd >= 0;
    if (!creator) {
      if (errno != EEXIST) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
    }
    if (creator) {
      if (cache_cap < 1) cache_cap = 1;   // maxsize 0 is enforced by the caller
      uint32_t nb = 1;
      while (nb < 2 * cache_cap) nb <<= 1;
      uint32_t lc = 1024;
      while (lc < lim_cap) lc <<= 1;
      const uint64_t eb = (sizeof(Entry) + value_max + 7) / 8 * 8;
      const uint64_t total = sizeof(Header) + (uint64_t)nb * 4 + eb * cache_cap + (uint64_t)lc * sizeof(Slot);
      if (ftruncate(fd, (off_t)total) != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("ftruncate: " + std::string(std::strerror(errno)));
      }
      s.map(fd, total);
      Header* h = s.h_;
      std::memset(static_cast<void*>(h), 0, sizeof(Header));
      h->version = kVersion;
      h->cache_cap = cache_cap;
      h->value_max = value_max;
      h->nbuckets = nb;
      h->lim_cap = lc;
      h->entry_bytes = eb;
      h->total_bytes = total;
      pthread_mutexattr_t at;
      pthread_mutexattr_init(&at);
      pthread_mutexattr_setpshared(&at, PTHREAD_PROCESS_SHARED);
      pthread_mutexattr_setrobust(&at, PTHREAD_MUTEX_ROBUST);
      pthread_mutex_init(&h->mu, &at);
      pthread_mutexattr_destroy(&at);
      s.reset_locked();
      __atomic_store_n(&h->magic, kMagic, __ATOMIC_RELEASE);   // published last: attachers wait for it
    } else {
      struct stat st;
      for (int i = 0; i < 2000; ++i) {   // the creator may still be sizing / initialising it
        if (fstat(fd, &st) == 0 && st.st_size >= (off_t)sizeof(Header)) break;
        usleep(1000);
      }
      if (st.st_size < (off_t)sizeof(Header)) {
        close(fd);
        throw std::runtime_error("shared state " + name + " was never initialised");
      }
      s.map(fd, (uint64_t)st.st_size);
      for (int i = 0; i < 2000 && __atomic_load_n(&s.h_->magic, __ATOMIC_ACQUIRE) != kMagic; ++i) usleep(1000);
      if (s.h_->magic != kMagic || s.h_->version != kVersion || s.h_->total_bytes != (uint64_t)st.st_size ||
          s.h_->value_max != value_max || s.h_->cache_cap != (cache_cap < 1 ? 1 : cache_cap))
        throw std::runtime_error("shared state " + name + " has an incompatible layout");
    }
    close(fd);
    return s;
  }

  SharedState() = default;
  SharedState(const SharedState&) = delete;
  SharedState& operator=(const SharedState&) = delete;
  SharedState(SharedState&& o) noexcept { *this = std::move(o); }
  SharedState& operator=(SharedState&& o) noexcept {
    std::swap(base_, o.base_);
    std::swap(bytes_, o.bytes_);
    std::swap(h_, o.h_);
    std::swap(name_, o.name_);
    return *this;
  }
  ~SharedState() {
    if (base_) munmap(base_, bytes_);
  }

  static void unlink(const std::string& name) { shm_unlink(name.c_str()); }
  const std::string& name() const { return name_; }
  uint32_t cache_capacity() const { return h_->cache_cap; }
  uint32_t value_max() const { return h_->value_max; }

  // ---- DP routing load -----------------------------------------------------------------------
  void load_set(uint32_t worker, uint32_t replica, int64_t v) {
    if (worker < kMaxWorkers && replica < kMaxReplicas) __atomic_store_n(&h_->load[worker][replica], v, __ATOMIC_RELAXED);
  }
  void load_clear_worker(uint32_t worker) {
    if (worker >= kMaxWorkers) return;
    for (uint32_t r = 0; r < kMaxReplicas; ++r) __atomic_store_n(&h_->load[worker][r], 0, __ATOMIC_RELAXED);
  }
  int64_t load_total(uint32_t replica) const {
    int64_t t = 0;
    if (replica >= kMaxReplicas) return 0;
    for (uint32_t w = 0; w < kMaxWorkers; ++w) t += __atomic_load_n(&h_->load[w][replica], __ATOMIC_RELAXED);
    return t;
  }
  // the live replica (bit r of live_mask) with the least total in-flight load; ties: lowest index.
  // -1 when none is live.
  int32_t load_pick(uint32_t n, uint64_t live_mask) const {
    int32_t best = -1;
    int64_t bl = 0;
    for (uint32_t r = 0; r < n && r < kMaxReplicas; ++r) {
      if (!((live_mask >> r) & 1u)) continue;
      const int64_t t = load_total(r);
      if (best < 0 || t < bl) {
        best = (int32_t)r;
        bl = t;
      }
    }
    return best;
  }

  // ---- cache -------------------------------------------------------------------------------
  // get: live value -> true (and the entry becomes most recently used); expired / absent -> false
  bool cache_get(uint64_t k0, uint64_t k1, double now, std::string* out, bool count_stats = true) {
    Lock l(this);
    const int32_t e = find(k0, k1);
    if (e < 0 || !(now < entry(e)->expires)) {
      if (count_stats) h_->misses++;
      return false;
    }
    lru_unlink(e);
    lru_push_back(e);
    if (count_stats) h_->hits++;
    if (out) out->assign(value(e), entry(e)->vlen);
    return true;
  }

  // set: stamp expires = now + ttl, make MRU; purge expired; evict LRU while full.  Returns false
  // (nothing stored) when the value does not fit the slot.
  bool cache_set(uint64_t k0, uint64_t k1, const std::string& v, double now, double ttl, uint32_t maxsize) {
    if (v.size() > h_->value_max) return false;
    Lock l(this);
    purge_expired(now);
    if (maxsize > h_->cache_cap) maxsize = h_->cache_cap;
    int32_t e = find(k0, k1);
    if (e < 0) {
      while (h_->count >= maxsize && h_->lru_head >= 0) evict(h_->lru_head);
      e = h_->free_head;
      if (e < 0) return false;   // unreachable: count < cap implies a free entry
      h_->free_head = entry(e)->next;
      Entry* en = entry(e);
      en->k0 = k0;
      en->k1 = k1;
      const uint32_t b = bucket(k0);
      en->hnext = buckets()[b];
      buckets()[b] = e;
      h_->count++;
    } else {
      lru_unlink(e);
    }
    Entry* en = entry(e);
    en->expires = now + ttl;
    en->vlen = (uint32_t)v.size();
    std::memcpy(value(e), v.data(), v.size());
    lru_push_back(e);
    h_->sets++;
    return true;
  }

  bool cache_delete(uint64_t k0, uint64_t k1) {
    Lock l(this);
    const int32_t e = find(k0, k1);
    if (e < 0) return false;
    remove(e);
    return true;
  }

  uint32_t cache_len(double now) {
    Lock l(this);
    uint32_t n = 0;
    for (int32_t e = h_->lru_head; e >= 0; e = entry(e)->next) n += now < entry(e)->expires;
    return n;
  }

  void cache_clear() {
    Lock l(this);
    while (h_->lru_head >= 0) remove(h_->lru_head);
  }

  // fault injection (tests): die holding the lock, half-way through a mutation
  [[noreturn]] void debug_die_locked(int code) {
    pthread_mutex_lock(&h_->mu);
    h_->lru_head = 0;   // a dangling chain: what an interrupted relink leaves behind
    _exit(code);
  }

  void stats(uint64_t* out) {   // hits, misses, sets, evictions, count, limiter slots used, owner deaths
    Lock l(this);
    out[0] = h_->hits;
    out[1] = h_->misses;
    out[2] = h_->sets;
    out[3] = h_->evictions;
    out[4] = h_->count;
    out[5] = h_->lim_used;
    out[6] = h_->owner_deaths;
  }

  // ---- fixed-window limiter (limits.FixedWindowRateLimiter.hit on a memory storage) -------------
  // The window starts at the first hit of the key and lasts `expiry` seconds; every hit counts
  // (also over the limit).  Returns true while count <= amount.
  bool limiter_hit(uint64_t k0, uint64_t k1, uint32_t amount, double expiry, double now) {
    Lock l(this);
    if (h_->lim_used * 4 >= (uint64_t)h_->lim_cap * 3) lim_rebuild(now);
    const uint32_t mask = h_->lim_cap - 1;
    uint32_t i = (uint32_t)(k0 ^ (k1 >> 17)) & mask;
    int64_t reuse = -1;
    for (uint32_t probe = 0; probe < h_->lim_cap; ++probe, i = (i + 1) & mask) {
      Slot* s = slot(i);
      if (s->state == 0) break;
      if (s->k0 == k0 && s->k1 == k1) {
        if (s->window_end <= now) {
          s->count = 0;
          s->window_end = now + expiry;
        }
        s->count++;
        return s->count <= amount;
      }
      if (reuse < 0 && s->window_end <= now) reuse = i;
    }
    Slot* s;
    if (reuse >= 0) {
      s = slot((uint32_t)reuse);
    } else {
      s = slot(i);
      if (s->state != 0) {   // table full of live windows: rebuild made room or we refuse to count
        lim_rebuild(now);
        return limiter_hit_unlocked_retry(k0, k1, amount, expiry, now);
      }
      s->state = 1;
      h_->lim_used++;
    }
    s->k0 = k0;
    s->k1 = k1;
    s->window_end = now + expiry;
    s->count = 1;
    return 1 <= amount;
  }

  void limiter_reset() {
    Lock l(this);
    std::memset(static_cast<void*>(slot(0)), 0, (size_t)h_->lim_cap * sizeof(Slot));
    h_->lim_used = 0;
  }

 private:
  struct Lock {
    Header* h;
    explicit Lock(SharedState* s) : h(s->h_) {
      const int rc = pthread_mutex_lock(&h->mu);
      if (rc == EOWNERDEAD) {
        // a worker died holding the lock, possibly half-way through relinking the LRU / hash chains:
        // nothing in the structures can be trusted, so start over (cache and limiter windows empty,
        // what a restart of the reference's single process would leave) before making it consistent
        s->reset_locked();
        ++h->owner_deaths;
        pthread_mutex_consistent(&h->mu);
      } else if (rc != 0) {
        throw std::runtime_error("shared state lock failed");
      }
    }
    ~Lock() { pthread_mutex_unlock(&h->mu); }
  };

  void map(int fd, uint64_t bytes) {
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) {
      close(fd);
      throw std::runtime_error("mmap: " + std::string(std::strerror(errno)));
    }
    base_ = static_cast<char*>(p);
    bytes_ = bytes;
    h_ = reinterpret_cast<Header*>(base_);
  }

  int32_t* buckets() const { return reinterpret_cast<int32_t*>(base_ + sizeof(Header)); }
  Entry* entry(int32_t e) const {
    return reinterpret_cast<Entry*>(base_ + sizeof(Header) + (uint64_t)h_->nbuckets * 4 + (uint64_t)e * h_->entry_bytes);
  }
  char* value(int32_t e) const { return reinterpret_cast<char*>(entry(e)) + sizeof(Entry); }
  Slot* slot(uint32_t i) const {
    return reinterpret_cast<Slot*>(base_ + sizeof(Header) + (uint64_t)h_->nbuckets * 4 +
                                   (uint64_t)h_->cache_cap * h_->entry_bytes) + i;
  }
  uint32_t bucket(uint64_t k0) const { return (uint32_t)(k0 ^ (k0 >> 29)) & (h_->nbuckets - 1); }

  void reset_locked() {
    for (uint32_t b = 0; b < h_->nbuckets; ++b) buckets()[b] = -1;
    for (uint32_t e = 0; e < h_->cache_cap; ++e) {
      Entry* en = entry((int32_t)e);
      std::memset(static_cast<void*>(en), 0, sizeof(Entry));
      en->next = e + 1 < h_->cache_cap ? (int32_t)e + 1 : -1;
      en->prev = en->hnext = -1;
    }
    h_->free_head = 0;
    h_->lru_head = h_->lru_tail = -1;
    h_->count = 0;
    std::memset(static_cast<void*>(slot(0)), 0, (size_t)h_->lim_cap * sizeof(Slot));
  }

  int32_t find(uint64_t k0, uint64_t k1) const {
    for (int32_t e = buckets()[bucket(k0)]; e >= 0; e = entry(e)->hnext)
      if (entry(e)->k0 == k0 && entry(e)->k1 == k1) return e;
    return -1;
  }
  void lru_unlink(int32_t e) {
    Entry* en = entry(e);
    if (en->prev >= 0) entry(en->prev)->next = en->next; else h_->lru_head = en->next;
    if (en->next >= 0) entry(en->next)->prev = en->prev; else h_->lru_tail = en->prev;
    en->prev = en->next = -1;
  }
  void lru_push_back(int32_t e) {
    Entry* en = entry(e);
    en->prev = h_->lru_tail;
    en->next = -1;
    if (h_->lru_tail >= 0) entry(h_->lru_tail)->next = e; else h_->lru_head = e;
    h_->lru_tail = e;
  }
  void remove(int32_t e) {
    lru_unlink(e);
    Entry* en = entry(e);
    int32_t* p = &buckets()[bucket(en->k0)];
    while (*p != e) p = &entry(*p)->hnext;
    *p = en->hnext;
    en->hnext = -1;
    en->next = h_->free_head;
    h_->free_head = e;
    h_->count--;
  }
  void evict(int32_t e) {
    remove(e);
    h_->evictions++;
  }
  void purge_expired(double now) {
    for (int32_t e = h_->lru_head; e >= 0;) {
      const int32_t nx = entry(e)->next;
      if (!(now < entry(e)->expires)) remove(e);
      e = nx;
    }
  }

  // drop expired windows and re-insert the live ones into a cleared table (restores the probe
  // chains without tombstones)
  void lim_rebuild(double now) {
    const uint32_t cap = h_->lim_cap, mask = cap - 1;
    std::vector<Slot> live;
    for (uint32_t i = 0; i < cap; ++i) {
      Slot* s = slot(i);
      if (s->state && s->window_end > now) live.push_back(*s);
    }
    std::memset(static_cast<void*>(slot(0)), 0, (size_t)cap * sizeof(Slot));
    for (const Slot& t : live) {
      uint32_t j = (uint32_t)(t.k0 ^ (t.k1 >> 17)) & mask;
      while (slot(j)->state) j = (j + 1) & mask;
      *slot(j) = t;
    }
    h_->lim_used = (uint64_t)live.size();
  }
  bool limiter_hit_unlocked_retry(uint64_t k0, uint64_t k1, uint32_t amount, double expiry, double now) {
    const uint32_t mask = h_->lim_cap - 1;
    uint32_t i = (uint32_t)(k0 ^ (k1 >> 17)) & mask;
    for (uint32_t probe = 0; probe < h_->lim_cap; ++probe, i = (i + 1) & mask) {
      Slot* s = slot(i);
      if (s->state == 0) {
        s->state = 1;
        s->k0 = k0;
        s->k1 = k1;
        s->window_end = now + expiry;
        s->count = 1;
        h_->lim_used++;
        return 1 <= amount;
      }
    }
    return false;   // every slot holds a live window: refuse (fail closed) rather than not count
  }

  char* base_ = nullptr;
  uint64_t bytes_ = 0;
  Header* h_ = nullptr;
  std::string name_;
};

}  // namespace ka
