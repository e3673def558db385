// checkpoint.cpp — ViT checkpoint files (include/vit_checkpoint.h), host-only code.
//
// Format: the llm.c convention of ViT::build_from_checkpoint (/root/reference/train_vit.rs:
// 89-143: 256-int header at byte 0, fp32 type-major parameters at byte 1024) completed with the
// ViT tensors and an optional AdamW state; see the header file for the field table.
#include <fcntl.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vit_checkpoint.h"

namespace vit {
void set_error(const char* fmt, ...);
}
using vit::set_error;

namespace {

struct File {
    FILE* f = nullptr;
    explicit File(FILE* f_) : f(f_) {}
    ~File() {
        if (f) fclose(f);
    }
};

bool config_ok(const vit_config_t& c) {
    return c.img > 0 && c.patch > 0 && c.img % c.patch == 0 && c.in_ch > 0 && c.channels > 0 &&
           c.num_layers > 0 && c.num_heads > 0 && c.channels % c.num_heads == 0 &&
           c.num_classes > 0;
}

uint32_t fbits(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return u;
}
float bitsf(uint32_t u) {
    float x;
    memcpy(&x, &u, 4);
    return x;
}

bool write_all(FILE* f, const void* p, size_t bytes) { return fwrite(p, 1, bytes, f) == bytes; }
bool read_all(FILE* f, void* p, size_t bytes) { return fread(p, 1, bytes, f) == bytes; }

}  // namespace

extern "C" {

long long vit_config_num_params(const vit_config_t* cfg) {
    if (!cfg || !config_ok(*cfg)) return 0;
    const long long C = cfg->channels, L = cfg->num_layers, NC = cfg->num_classes;
    const long long np = (long long)(cfg->img / cfg->patch) * (cfg->img / cfg->patch);
    const long long K = (long long)cfg->in_ch * cfg->patch * cfg->patch, T = np + 1;
    // the 20 canonical tensors (vit_trainer.h): embed, 12 per-layer kinds, lnf, head
    return C * K + C + C + T * C + L * (C + C + 3 * C * C + 3 * C + C * C + C + C + C +
                                        4 * C * C + 4 * C + 4 * C * C + C) +
           C + C + NC * C + NC;
}

int vit_checkpoint_read_info(const char* path, vit_checkpoint_info_t* info) {
    if (!path || !info) {
        set_error("vit_checkpoint_read_info: null argument");
        return 1;
    }
    File fh(fopen(path, "rb"));
    if (!fh.f) {
        set_error("checkpoint %s: cannot open", path);
        return 1;
    }
    int32_t h[256];
    if (!read_all(fh.f, h, sizeof(h))) {
        set_error("checkpoint %s: short header", path);
        return 1;
    }
    if (h[0] != VIT_CKPT_MAGIC || h[1] != VIT_CKPT_VERSION) {
        set_error("checkpoint %s: bad magic/version %d/%d", path, h[0], h[1]);
        return 1;
    }
    vit_checkpoint_info_t in{};
    in.cfg.num_classes = h[3];
    in.cfg.num_layers = h[4];
    in.cfg.num_heads = h[5];
    in.cfg.channels = h[6];
    in.cfg.img = h[7];
    in.cfg.patch = h[8];
    in.cfg.in_ch = h[9];
    in.has_opt = h[10] & 1;
    in.step = h[11];
    in.num_params = (long long)(uint32_t)h[12] | ((long long)(uint32_t)h[13] << 32);
    in.adamw = {bitsf((uint32_t)h[14]), bitsf((uint32_t)h[15]), bitsf((uint32_t)h[16]),
                bitsf((uint32_t)h[17])};
    if (!config_ok(in.cfg)) {
        set_error("checkpoint %s: invalid config in header", path);
        return 1;
    }
    const long long np = (long long)(in.cfg.img / in.cfg.patch) * (in.cfg.img / in.cfg.patch);
    if (h[2] != np + 1) {
        set_error("checkpoint %s: max_seq_len %d != (img/patch)^2+1 = %lld", path, h[2], np + 1);
        return 1;
    }
    if (in.num_params != vit_config_num_params(&in.cfg)) {
        set_error("checkpoint %s: num_params %lld does not match the config (%lld)", path,
                  in.num_params, vit_config_num_params(&in.cfg));
        return 1;
    }
    if (fseeko(fh.f, 0, SEEK_END) != 0) {
        set_error("checkpoint %s: seek failed", path);
        return 1;
    }
    const long long want = VIT_CKPT_HEADER_BYTES + in.num_params * 4 * (in.has_opt ? 3 : 1);
    const long long have = (long long)ftello(fh.f);
    if (have != want) {
        set_error("checkpoint %s: %lld bytes, expected %lld", path, have, want);
        return 1;
    }
    *info = in;
    return 0;
}

int vit_checkpoint_write(const char* path, const vit_config_t* cfg, const float* params,
                         const float* m, const float* v, int step, const vit_adamw_t* adamw) {
    if (!path || !cfg || !params || (!m) != (!v)) {
        set_error("vit_checkpoint_write: bad arguments");
        return 1;
    }
    if (!config_ok(*cfg)) {
        set_error("vit_checkpoint_write: invalid config");
        return 1;
    }
    const long long n = vit_config_num_params(cfg);
    const int np = (cfg->img / cfg->patch) * (cfg->img / cfg->patch);
    std::vector<int32_t> hdr(VIT_CKPT_HEADER_BYTES / 4, 0);
    hdr[0] = VIT_CKPT_MAGIC;
    hdr[1] = VIT_CKPT_VERSION;
    hdr[2] = np + 1;
    hdr[3] = cfg->num_classes;
    hdr[4] = cfg->num_layers;
    hdr[5] = cfg->num_heads;
    hdr[6] = cfg->channels;
    hdr[7] = cfg->img;
    hdr[8] = cfg->patch;
    hdr[9] = cfg->in_ch;
    hdr[10] = m ? 1 : 0;
    hdr[11] = m ? step : 0;
    hdr[12] = (int32_t)(uint32_t)(n & 0xffffffffLL);
    hdr[13] = (int32_t)(uint32_t)(n >> 32);
    if (m && adamw) {
        hdr[14] = (int32_t)fbits(adamw->beta1);
        hdr[15] = (int32_t)fbits(adamw->beta2);
        hdr[16] = (int32_t)fbits(adamw->eps);
        hdr[17] = (int32_t)fbits(adamw->weight_decay);
    }
    // write to path.tmp and rename, so an interrupted save never leaves a truncated checkpoint
    const std::string tmp = std::string(path) + ".tmp";
    {
        File fh(fopen(tmp.c_str(), "wb"));
        if (!fh.f) {
            set_error("checkpoint %s: cannot create", tmp.c_str());
            return 1;
        }
        bool ok = write_all(fh.f, hdr.data(), VIT_CKPT_HEADER_BYTES) &&
                  write_all(fh.f, params, (size_t)n * 4);
        if (ok && m) ok = write_all(fh.f, m, (size_t)n * 4) && write_all(fh.f, v, (size_t)n * 4);
        // durable before the rename: the data blocks must reach the disk before the new name does
        ok = ok && fflush(fh.f) == 0 && fsync(fileno(fh.f)) == 0;
        if (!ok) {
            set_error("checkpoint %s: write failed", tmp.c_str());
            fclose(fh.f);
            fh.f = nullptr;
            remove(tmp.c_str());
            return 1;
        }
    }
    if (rename(tmp.c_str(), path) != 0) {
        set_error("checkpoint %s: rename failed", path);
        remove(tmp.c_str());
        return 1;
    }
    // and the rename itself: fsync the directory entry
    std::string dir(path);
    const size_t slash = dir.find_last_of('/');
    dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : dir.substr(0, slash));
    const int dfd = open(dir.c_str(), O_RDONLY | O_DIRECTORY);
    if (dfd >= 0) {
        fsync(dfd);
        close(dfd);
    }
    return 0;
}

int vit_checkpoint_read(const char* path, const vit_config_t* cfg, float* params, float* m,
                        float* v) {
    vit_checkpoint_info_t in;
    if (vit_checkpoint_read_info(path, &in)) return 1;
    if (!cfg || !params || memcmp(&in.cfg, cfg, sizeof(vit_config_t)) != 0) {
        set_error("checkpoint %s: config differs from the model's", path);
        return 1;
    }
    File fh(fopen(path, "rb"));
    if (!fh.f || fseeko(fh.f, VIT_CKPT_HEADER_BYTES, SEEK_SET) != 0 ||
        !read_all(fh.f, params, (size_t)in.num_params * 4)) {
        set_error("checkpoint %s: short parameter section", path);
        return 1;
    }
    if (in.has_opt && (m || v)) {
        bool ok = m ? read_all(fh.f, m, (size_t)in.num_params * 4)
                    : fseeko(fh.f, in.num_params * 4, SEEK_CUR) == 0;
        if (ok && v) ok = read_all(fh.f, v, (size_t)in.num_params * 4);
        if (!ok) {
            set_error("checkpoint %s: short optimizer section", path);
            return 1;
        }
    }
    return 0;
}

}  // extern "C"
