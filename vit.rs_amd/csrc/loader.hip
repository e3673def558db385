// loader.hip — native record loader of the input pipeline (include/vit_data.h).
// Host code only (no kernels): mmap'd uint8 HWC records, a seeded per-epoch shuffle, the batch of
// each data-parallel rank, and a background thread that assembles batches into a ring of host
// buffers (page-locked via hipHostMalloc when asked, so the trainer's upload is a real async DMA).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/vit_data.h"

namespace vit {
void set_error(const char* fmt, ...);
}
using vit::set_error;

namespace {

// counter-form splitmix64: output i (0-based) = mix(seed + (i+1) * golden)  (data.py splitmix64)
inline uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct Mapped {
    void* p = MAP_FAILED;
    size_t bytes = 0;
    bool open(const char* path) {
        int fd = ::open(path, O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0 || st.st_size <= 0) {
            ::close(fd);
            return false;
        }
        bytes = (size_t)st.st_size;
        p = mmap(nullptr, bytes, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        return p != MAP_FAILED;
    }
    ~Mapped() {
        if (p != MAP_FAILED) munmap(p, bytes);
    }
};

}  // namespace

struct vit_loader {
    Mapped images, labels;
    long long N = 0;
    size_t rec_bytes = 0;
    int B = 0, rank = 0, world = 1, shuffle = 1, pinned = 0, depth = 3, steps = 0;
    uint64_t seed = 0;

    struct Slot {
        unsigned char* img = nullptr;
        int* lab = nullptr;
        long long epoch = 0;
        int step = 0;
        int state = 0;  // 0 free, 1 ready, 2 handed out
    };
    std::vector<Slot> slots;
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
    std::thread worker;
    size_t next_fill = 0, next_take = 0;
    long long out_slot = -1;
    std::vector<long long> perm;
    long long perm_epoch = -1;

    void make_perm(long long epoch) {
        perm.resize((size_t)N);
        for (long long i = 0; i < N; i++) perm[(size_t)i] = i;
        if (shuffle) {
            const uint64_t s = seed + (uint64_t)epoch;
            for (long long i = N - 1; i >= 1; i--) {
                const uint64_t r = splitmix64_at(s, (uint64_t)(N - 1 - i));
                std::swap(perm[(size_t)i], perm[(size_t)(r % (uint64_t)(i + 1))]);
            }
        }
        perm_epoch = epoch;
    }

    void fill(Slot& sl, long long seq) {
        const long long epoch = seq / steps;
        const int step = (int)(seq % steps);
        if (epoch != perm_epoch) make_perm(epoch);
        const long long base = ((long long)step * world + rank) * B;
        const unsigned char* src = (const unsigned char*)images.p;
        const int* lsrc = (const int*)labels.p;
        for (int b = 0; b < B; b++) {
            const long long r = perm[(size_t)(base + b)];
            memcpy(sl.img + (size_t)b * rec_bytes, src + (size_t)r * rec_bytes, rec_bytes);
            sl.lab[b] = lsrc[r];
        }
        sl.epoch = epoch;
        sl.step = step;
    }

    void run() {
        long long seq = 0;
        for (;;) {
            Slot* sl;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || slots[next_fill].state == 0; });
                if (stop) return;
                sl = &slots[next_fill];
            }
            fill(*sl, seq++);  // outside the lock: the slot is owned by the worker while free
            {
                std::lock_guard<std::mutex> lk(mu);
                sl->state = 1;
                next_fill = (next_fill + 1) % slots.size();
            }
            cv.notify_all();
        }
    }

    void free_slots() {
        for (auto& s : slots) {
            if (pinned) {
                if (s.img) (void)hipHostFree(s.img);
            } else {
                free(s.img);
            }
            free(s.lab);
        }
        slots.clear();
    }
};

extern "C" {

vit_loader_t* vit_loader_open(const char* images_path, const char* labels_path, int img,
                              int batch, unsigned long long seed, int rank, int world, int shuffle,
                              int pinned, int depth) {
    if (!images_path || !labels_path || img <= 0 || batch <= 0 || world < 1 || rank < 0 ||
        rank >= world || depth < 2) {
        set_error("vit_loader_open: bad arguments");
        return nullptr;
    }
    auto* l = new vit_loader();
    l->rec_bytes = (size_t)img * img * 3;
    if (!l->images.open(images_path) || !l->labels.open(labels_path)) {
        set_error("vit_loader_open: cannot map %s / %s", images_path, labels_path);
        delete l;
        return nullptr;
    }
    if (l->images.bytes % l->rec_bytes || l->labels.bytes % 4 ||
        (long long)(l->images.bytes / l->rec_bytes) != (long long)(l->labels.bytes / 4)) {
        set_error("vit_loader_open: %zu image bytes / %zu label bytes are not N records of %zu + 4",
                  l->images.bytes, l->labels.bytes, l->rec_bytes);
        delete l;
        return nullptr;
    }
    l->N = (long long)(l->labels.bytes / 4);
    l->B = batch;
    l->rank = rank;
    l->world = world;
    l->seed = seed;
    l->shuffle = shuffle != 0;
    l->pinned = pinned != 0;
    l->depth = depth;
    l->steps = (int)(l->N / ((long long)batch * world));
    if (l->steps < 1) {
        set_error("vit_loader_open: %lld records < one global batch of %d x %d", l->N, batch, world);
        delete l;
        return nullptr;
    }
    l->slots.resize((size_t)depth);
    for (auto& s : l->slots) {
        const size_t bytes = l->rec_bytes * (size_t)batch;
        if (l->pinned) {
            if (hipHostMalloc((void**)&s.img, bytes, hipHostMallocDefault) != hipSuccess) s.img = nullptr;
        } else {
            s.img = (unsigned char*)malloc(bytes);
        }
        s.lab = (int*)malloc(sizeof(int) * (size_t)batch);
        if (!s.img || !s.lab) {
            set_error("vit_loader_open: host allocation of %zu bytes failed", bytes);
            l->free_slots();
            delete l;
            return nullptr;
        }
    }
    l->worker = std::thread([l] { l->run(); });
    return l;
}

long long vit_loader_num_records(const vit_loader_t* l) { return l ? l->N : 0; }
int vit_loader_steps_per_epoch(const vit_loader_t* l) { return l ? l->steps : 0; }

int vit_loader_next(vit_loader_t* l, const unsigned char** images, const int** labels,
                    long long* epoch, int* step) {
    if (!l) {
        set_error("vit_loader_next: null loader");
        return 1;
    }
    std::unique_lock<std::mutex> lk(l->mu);
    if (l->out_slot >= 0) {  // the previous batch goes back to the worker
        l->slots[(size_t)l->out_slot].state = 0;
        l->out_slot = -1;
        l->cv.notify_all();
    }
    l->cv.wait(lk, [&] { return l->slots[l->next_take].state == 1; });
    auto& s = l->slots[l->next_take];
    s.state = 2;
    l->out_slot = (long long)l->next_take;
    l->next_take = (l->next_take + 1) % l->slots.size();
    if (images) *images = s.img;
    if (labels) *labels = s.lab;
    if (epoch) *epoch = s.epoch;
    if (step) *step = s.step;
    return 0;
}

void vit_loader_close(vit_loader_t* l) {
    if (!l) return;
    {
        std::lock_guard<std::mutex> lk(l->mu);
        l->stop = true;
    }
    l->cv.notify_all();
    if (l->worker.joinable()) l->worker.join();
    l->free_slots();
    delete l;
}

}  // extern "C"
