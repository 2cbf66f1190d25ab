// Host emulation runtime for tools_cpu/bdemu (see emu/hip/hip_runtime.h):
// a pool of lane threads, block and wave barriers, the wave exchange.
#include <barrier>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>

#include "hip/hip_runtime.h"

#if defined(__has_feature)
#if __has_feature(memory_sanitizer)
#include <sanitizer/msan_interface.h>
#define EMU_MSAN 1
#endif
#endif

thread_local emu_u3 threadIdx, blockIdx, blockDim, gridDim;

namespace emu {
namespace {

struct Wave {
    std::unique_ptr<std::barrier<>> bar;
    uint64_t slots[64];
    std::atomic<uint64_t> live{0};
};
struct Block {
    int nthreads = 0;
    std::unique_ptr<std::barrier<>> bar;
    std::vector<std::unique_ptr<Wave>> waves;
    dim3 bidx, grid, bdim;
    const std::function<void()>* body = nullptr;
    std::atomic<int> acc[3] = {0, 0, 0};  // __syncthreads_count slots, used in rotation
};

thread_local int t_lane = 0, t_wave = 0, t_sc = 0;
thread_local Block* t_block = nullptr;
thread_local uint64_t t_copy[64];
char* g_dyn = nullptr;
std::mutex g_lds_mu;
std::vector<std::pair<void*, size_t>> g_lds;
int lds_fill() {
    static const int f = getenv("EMU_LDS_FILL") ? (int)strtol(getenv("EMU_LDS_FILL"), nullptr, 0) : 0xA5;
    return f;
}

// A fixed pool of lane threads; a block runs on its first nthreads workers.
class Pool {
   public:
    static constexpr int kMax = 1024;
    Pool() {
        for (int i = 0; i < kMax; ++i) th_.emplace_back([this, i] { worker(i); });
    }
    void run(Block* b) {
        std::unique_lock<std::mutex> lk(mu_);
        job_ = b;
        pending_ = b->nthreads;
        ++gen_;
        cv_.notify_all();
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

   private:
    void worker(int id) {
        uint64_t seen = 0;
        for (;;) {
            Block* b;
            int nt;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                b = job_;
                nt = b ? b->nthreads : 0;  // b outlives only the job's own lanes
            }
            if (!b || id >= nt) continue;
            const unsigned bx = b->bdim.x, by = b->bdim.y;
            threadIdx.x = id % bx;
            threadIdx.y = (id / bx) % by;
            threadIdx.z = id / (bx * by);
            blockIdx.x = b->bidx.x;
            blockIdx.y = b->bidx.y;
            blockIdx.z = b->bidx.z;
            blockDim.x = b->bdim.x;
            blockDim.y = b->bdim.y;
            blockDim.z = b->bdim.z;
            gridDim.x = b->grid.x;
            gridDim.y = b->grid.y;
            gridDim.z = b->grid.z;
            t_lane = id & 63;
            t_wave = id >> 6;
            t_block = b;
            t_sc = 0;
            (*b->body)();
            Wave& w = *b->waves[t_wave];
            w.live.fetch_and(~(1ull << t_lane));
            w.bar->arrive_and_drop();
            b->bar->arrive_and_drop();
            t_block = nullptr;
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    Block* job_ = nullptr;
    int pending_ = 0;
    uint64_t gen_ = 0;
};

Pool& pool() {
    static Pool* p = new Pool();  // never joined: the process exits with the workers parked
    return *p;
}

}  // namespace

void launch(const Cfg& c, const char* name, const std::function<void()>& body) {
    const int nt = (int)(c.b.x * c.b.y * c.b.z);
    if (nt <= 0 || nt > Pool::kMax) {
        fprintf(stderr, "emu: %s: block of %d threads\n", name, nt);
        abort();
    }
    const uint64_t blocks = (uint64_t)c.g.x * c.g.y * c.g.z;
    if (getenv("EMU_TRACE"))
        fprintf(stderr, "emu: launch %s grid (%u,%u,%u) block %d shm %zu\n", name, c.g.x, c.g.y,
                c.g.z, nt, c.shm);
    std::vector<char> dyn(c.shm ? c.shm : 1);
    g_dyn = dyn.data();
    // a launch that never finishes (a wave operation some lanes skip, a
    // spin-wait on a later workgroup) is reported instead of hanging
    const unsigned budget = getenv("EMU_ALARM") ? (unsigned)atoi(getenv("EMU_ALARM")) : 120u;
    for (uint64_t i = 0; i < blocks; ++i) {
        Block b;
        b.nthreads = nt;
        b.bar = std::make_unique<std::barrier<>>(nt);
        const int nw = (nt + 63) / 64;
        for (int w = 0; w < nw; ++w) {
            auto wv = std::make_unique<Wave>();
            const int lanes = std::min(64, nt - 64 * w);
            wv->bar = std::make_unique<std::barrier<>>(lanes);
            wv->live = lanes == 64 ? ~0ull : ((1ull << lanes) - 1);
            memset(wv->slots, 0, sizeof(wv->slots));
            b.waves.push_back(std::move(wv));
        }
        b.bidx = dim3((unsigned)(i % c.g.x), (unsigned)((i / c.g.x) % c.g.y),
                      (unsigned)(i / ((uint64_t)c.g.x * c.g.y)));
        b.grid = c.g;
        b.bdim = c.b;
        b.body = &body;
        if (c.shm) memset(dyn.data(), lds_fill(), c.shm);  // undefined LDS content
        {
            std::lock_guard<std::mutex> lk(g_lds_mu);
            for (auto& r : g_lds) {
#ifdef EMU_MSAN
                __msan_poison(r.first, r.second);  // undefined at workgroup start
#else
                memset(r.first, lds_fill(), r.second);
#endif
            }
        }
        alarm(budget);
        pool().run(&b);
        alarm(0);
    }
    g_dyn = nullptr;
}

void lds_register(void* p, size_t n) {
    std::lock_guard<std::mutex> lk(g_lds_mu);
    g_lds.emplace_back(p, n);
}
void check_failed(const char* what, long long v, const char* file, int line) {
    fprintf(stderr, "emu: index check failed: %s = %lld at %s:%d (block %u,%u thread %u)\n", what, v,
            file, line, blockIdx.x, blockIdx.y, threadIdx.x);
    abort();
}

void syncthreads() { t_block->bar->arrive_and_wait(); }
int syncthreads_count(int p) {
    std::atomic<int>& a = t_block->acc[t_sc++ % 3];
    a.fetch_add(p ? 1 : 0);
    t_block->bar->arrive_and_wait();
    const int r = a.load();
    t_block->bar->arrive_and_wait();
    if (threadIdx.x == 0 && threadIdx.y == 0 && threadIdx.z == 0) a.store(0);
    return r;
}
int lane() { return t_lane; }
int wave_size() { return 64; }
void* dyn_lds() { return g_dyn; }
void fence() { std::atomic_thread_fence(std::memory_order_seq_cst); }

const uint64_t* wave_exchange(uint64_t v, uint64_t* live) {
    Wave& w = *t_block->waves[t_wave];
    w.slots[t_lane] = v;
    w.bar->arrive_and_wait();
    memcpy(t_copy, w.slots, sizeof(t_copy));
    if (live) *live = w.live.load();
    w.bar->arrive_and_wait();
    return t_copy;
}

}  // namespace emu
