// Host-side mirror of the reference's `path` plugin (MIPathTracer,
// src/integrators/path/path.cpp) whose render() drives the GPU library
// instead of the per-sample CPU loop of SamplingIntegrator::render
// (src/librender/integrator.cpp:99-133): one host thread per GPU, each
// renders a share of the 16x16 film tiles (balanced from the last render's
// rates, see mtsh_path_job_render) into its own
// ImageBlock (tile rect + border), and the blocks are merged by addition
// exactly like ImageBlock::put(const ImageBlock*) (imageblock.h:103-107).
// No collectives: the film is the only thing exchanged (host-side gather).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtsg.h"
#include "../../include/mtsh.h"
#include "../../include/mtsg_path.h"

namespace {
thread_local std::string g_perr;

std::string device_error() {
    char buf[1024];
    mtsg_last_error(buf, sizeof(buf));
    return buf;
}
}  // namespace

struct mtsh_path_job {
    std::vector<mtsg_scene *> handles;
    int border = 0;
    // cancel(): the job's flag is checked by each worker before its render
    // starts; the handles' flags stop renders already running (per bounce)
    std::atomic<int> cancel{0};
    // per GPU, under gpuLock[g]: its mtsg_render is running, and a cancel was
    // sent to it.  A cancel that reaches the handle after its render returned
    // would stay set and cancel the job's next render, so the worker withdraws
    // it (mtsg_cancel_clear) when its render is over; the lock orders the two.
    std::vector<int> rendering, sent;
    std::vector<std::mutex> gpuLock;
    std::mutex renderLock;   // one render at a time per job
    // tile completion: the caller's hook, serialised over the GPU threads
    mtsh_path_tile_fn tileFn = nullptr;
    void *tileUser = nullptr;
    std::mutex tileLock;
    struct TileCtx { mtsh_path_job *job; int gpu; };
    std::vector<TileCtx> tileCtx;
    // share balancing (mtsh_path_job_set_balance): the last render's tiles
    // and seconds per GPU, for the next render of the same tile set
    int balance = 1;
    std::vector<int> lastCount;
    std::vector<double> lastSec;
    std::vector<int64_t> lastSig;
    // the largest share each GPU has rendered: a render past it may have
    // (re)allocated the handle's batch buffers, so its time is not a rate
    std::vector<size_t> maxShare;
    explicit mtsh_path_job(int n) : rendering(n, 0), sent(n, 0), gpuLock(n), maxShare(n, 0) {}
};

namespace {
void tile_trampoline(void *user, int32_t, int32_t x, int32_t y, int32_t w, int32_t h) {
    auto *c = static_cast<mtsh_path_job::TileCtx *>(user);
    std::lock_guard<std::mutex> lock(c->job->tileLock);
    if (c->job->tileFn) c->job->tileFn(c->job->tileUser, c->gpu, x, y, w, h);
}
// The caller's tiles in the order balanced shares are cut from: deal key k
// at position frac(k * golden ratio), so a run of any length is spread over
// the whole rectangle (mtsg.balance_order is the same order)
std::vector<int32_t> balance_order(const std::vector<int32_t> &keys) {
    const double phi = (std::sqrt(5.0) - 1.0) / 2.0;
    std::vector<std::pair<double, int32_t>> o;
    o.reserve(keys.size());
    for (int32_t k : keys) {
        double ip;
        o.emplace_back(std::modf((double)k * phi, &ip), k);
    }
    std::stable_sort(o.begin(), o.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::vector<int32_t> out;
    out.reserve(o.size());
    for (auto &e : o) out.push_back(e.second);
    return out;
}

// next tile counts from the last render (mtsg.balance_cuts): GPU g took
// sec[g] for count[g] tiles, so it is given count[g] / sec[g] of the total,
// mixed half and half with its old count; every GPU keeps at least one tile
std::vector<int> balance_cuts(const std::vector<int> &count, const std::vector<double> &sec) {
    const size_t n = count.size();
    double total = 0, rsum = 0;
    for (size_t g = 0; g < n; ++g) {
        total += count[g];
        rsum += count[g] / std::max(sec[g], 1e-9);
    }
    std::vector<double> want(n);
    std::vector<int> out(n);
    long sum = 0;
    for (size_t g = 0; g < n; ++g) {
        const double target = count[g] / std::max(sec[g], 1e-9) / rsum * total;
        want[g] = 0.5 * count[g] + 0.5 * target;
        out[g] = std::max(1, (int)std::floor(want[g]));
        sum += out[g];
    }
    std::vector<size_t> order(n);
    for (size_t g = 0; g < n; ++g) order[g] = g;
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t a, size_t b) { return want[a] - std::floor(want[a]) > want[b] - std::floor(want[b]); });
    long rest = (long)std::llround(total) - sum;
    for (size_t k = 0; rest != 0 && k < 4 * n + (size_t)std::labs(rest) * n; ++k) {
        const size_t g = order[k % n];
        if (rest > 0) { ++out[g]; --rest; }
        else if (out[g] > 1) { --out[g]; ++rest; }
    }
    return out;
}
}  // namespace

extern "C" {

int mtsh_path_job_create(const mtsh_scene *scene, int n_gpus, mtsh_path_job **out) {
    if (!scene || !out) { g_perr = "null argument"; return MTSG_ERR_INVALID; }
    *out = nullptr;
    const int avail = mtsg_device_count();
    if (n_gpus <= 0) n_gpus = avail;
    if (n_gpus > avail || n_gpus <= 0) {
        g_perr = "requested " + std::to_string(n_gpus) + " GPU(s), " + std::to_string(avail) + " gfx950 device(s) visible";
        return MTSG_ERR_NODEVICE;
    }
    const mtsg_scene_desc *desc = mtsh_scene_desc(scene);
    mtsh_scene_info info;
    mtsh_scene_get_info(scene, &info);
    auto *job = new mtsh_path_job(n_gpus);
    job->border = info.border;
    job->handles.assign(n_gpus, nullptr);
    // upload (preprocessing; excluded from the render time like renderjob.cpp:102)
    for (int g = 0; g < n_gpus; ++g) {
        const int rc = mtsg_scene_create(desc, g, &job->handles[g]);
        if (rc != MTSG_OK) {
            g_perr = "GPU " + std::to_string(g) + ": " + device_error();
            mtsh_path_job_destroy(job);
            return rc;
        }
    }
    *out = job;
    return MTSG_OK;
}

int mtsh_path_job_gpus(const mtsh_path_job *job) { return job ? (int)job->handles.size() : 0; }

int mtsh_path_job_set_tile_callback(mtsh_path_job *job, mtsh_path_tile_fn fn, void *user) {
    if (!job) { g_perr = "null argument"; return MTSG_ERR_INVALID; }
    std::lock_guard<std::mutex> lock(job->renderLock);   // not while a render runs
    {
        std::lock_guard<std::mutex> tl(job->tileLock);
        job->tileFn = fn;
        job->tileUser = user;
    }
    job->tileCtx.resize(job->handles.size());
    for (size_t g = 0; g < job->handles.size(); ++g) {
        job->tileCtx[g] = {job, (int)g};
        mtsg_set_tile_callback(job->handles[g], fn ? tile_trampoline : nullptr, fn ? &job->tileCtx[g] : nullptr);
    }
    return MTSG_OK;
}

int mtsh_path_job_render(mtsh_path_job *job, const mtsg_render_params *params, float *rgbaw_out,
                         double *seconds_out) {
    if (!job || !params || !rgbaw_out) { g_perr = "null argument"; return MTSG_ERR_INVALID; }
    std::lock_guard<std::mutex> lock(job->renderLock);
    const int n = (int)job->handles.size();
    const int b = job->border;
    if (params->tile_w <= 0 || params->tile_h <= 0) { g_perr = "tile rectangle outside the film"; return MTSG_ERR_INVALID; }
    if (params->tile_stride < 0 || (params->tile_stride > 1 && (params->tile_offset < 0 || params->tile_offset >= params->tile_stride))) {
        g_perr = "invalid tile_stride / tile_offset";
        return MTSG_ERR_INVALID;
    }
    const size_t W = (size_t)params->tile_w + 2 * b, H = (size_t)params->tile_h + 2 * b;
    // the caller's tile subset: deal keys off + k * S of the rectangle's tiles
    const int S = params->tile_stride > 1 ? params->tile_stride : 1;
    const int off = params->tile_stride > 1 ? params->tile_offset : 0;
    const int allTiles = ((params->tile_w + 15) / 16) * ((params->tile_h + 15) / 16);
    std::vector<int32_t> keys;
    for (int k = off; k < allTiles; k += S) keys.push_back(k);
    // Shares.  A GPU renders its share as one wavefront batch, so handing out
    // tile groups from a queue during the render (the reference scheduler's
    // acquireWork, src/libcore/sched.cpp:427-496) would cut the share into
    // batches that each pay the per-bounce launch drain;
    // instead each GPU takes a run of the golden-ratio key order, and a render
    // of the same tile set as the last one re-cuts the runs from the GPUs'
    // measured rates (balance_cuts).  Any cut gives the same image: the
    // random numbers are keyed by pixel and sample.
    const std::vector<int64_t> sig = {params->tile_x, params->tile_y, params->tile_w, params->tile_h, S, off,
                                      (int64_t)params->spp, params->max_depth, params->integrator};
    std::vector<int> count(n, 0);
    if (job->balance && n > 1 && job->lastSig == sig && (int)job->lastCount.size() == n &&
        (int)keys.size() >= n) {
        count = balance_cuts(job->lastCount, job->lastSec);
    } else {
        for (int g = 0; g < n; ++g) count[g] = (int)(keys.size() / n + ((size_t)g < keys.size() % n ? 1 : 0));
    }
    const std::vector<int32_t> order = balance_order(keys);
    std::vector<std::vector<int32_t>> share(n);
    for (int g = 0, lo = 0; g < n; lo += count[g], ++g) {
        share[g].assign(order.begin() + lo, order.begin() + lo + count[g]);
        std::sort(share[g].begin(), share[g].end());
    }
    std::vector<std::vector<float>> blocks(n, std::vector<float>(W * H * 5));
    std::vector<int> rcs(n, MTSG_OK);
    std::vector<double> sec(n, 0.0);
    std::vector<std::string> errs(n);
    job->cancel.store(0);   // a cancel() while idle has no effect
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> threads;
    for (int g = 0; g < n; ++g)
        threads.emplace_back([&, g]() {
            mtsg_render_params p = *params;
            p.tile_stride = 1;
            p.tile_offset = 0;
            {
                std::lock_guard<std::mutex> gl(job->gpuLock[g]);
                job->rendering[g] = 1;
            }
            // the render call alone is timed (not the tile-list upload)
            if (job->cancel.load()) rcs[g] = MTSG_ERR_CANCELLED;
            else if (share[g].empty()) rcs[g] = MTSG_OK;   // fewer tiles than GPUs: this one idles
            else if ((rcs[g] = mtsg_set_tile_list(job->handles[g], share[g].data(), (uint32_t)share[g].size())) == MTSG_OK) {
                const auto tg = std::chrono::steady_clock::now();
                rcs[g] = mtsg_render(job->handles[g], &p, blocks[g].data());
                sec[g] = std::chrono::duration<double>(std::chrono::steady_clock::now() - tg).count();
            }
            {
                std::lock_guard<std::mutex> gl(job->gpuLock[g]);
                job->rendering[g] = 0;
                if (job->sent[g]) mtsg_cancel_clear(job->handles[g]);
                job->sent[g] = 0;
            }
            // the device library's error is thread-local: capture it here
            if (rcs[g] != MTSG_OK) errs[g] = device_error();
        });
    for (auto &t : threads) t.join();
    if (seconds_out) *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool cancelled = job->cancel.exchange(0) != 0;
    for (int g = 0; g < n; ++g)
        if (rcs[g] != MTSG_OK && rcs[g] != MTSG_ERR_CANCELLED) {
            g_perr = "GPU " + std::to_string(g) + ": " + errs[g];
            return rcs[g];
        }
    for (int g = 0; g < n; ++g)
        if (rcs[g] == MTSG_ERR_CANCELLED || cancelled) {
            g_perr = "cancelled";
            return MTSG_ERR_CANCELLED;
        }
    std::memset(rgbaw_out, 0, W * H * 5 * sizeof(float));
    for (int g = 0; g < n; ++g)
        for (size_t i = 0; i < W * H * 5; ++i) rgbaw_out[i] += blocks[g][i];
    // a GPU whose share grew past any it rendered before may have spent part
    // of its time allocating: that render keeps the cut (no re-cut from it)
    bool grew = false;
    for (int g = 0; g < n; ++g) {
        grew |= share[g].size() > job->maxShare[g];
        job->maxShare[g] = std::max(job->maxShare[g], share[g].size());
    }
    job->lastSig = grew ? std::vector<int64_t>() : sig;
    job->lastCount = count;
    job->lastSec = sec;
    return MTSG_OK;
}

int mtsh_path_job_set_balance(mtsh_path_job *job, int on) {
    if (!job) { g_perr = "null argument"; return MTSG_ERR_INVALID; }
    std::lock_guard<std::mutex> lock(job->renderLock);
    job->balance = on != 0;
    job->lastSig.clear();
    return MTSG_OK;
}

int mtsh_path_job_shares(const mtsh_path_job *job, int32_t *tiles, double *seconds) {
    if (!job) { g_perr = "null argument"; return MTSG_ERR_INVALID; }
    // not while a render of the job rewrites them
    std::lock_guard<std::mutex> lock(const_cast<mtsh_path_job *>(job)->renderLock);
    const size_t n = job->handles.size();
    for (size_t g = 0; g < n; ++g) {
        if (tiles) tiles[g] = g < job->lastCount.size() ? job->lastCount[g] : 0;
        if (seconds) seconds[g] = g < job->lastSec.size() ? job->lastSec[g] : 0.0;
    }
    return MTSG_OK;
}

void mtsh_path_job_cancel(mtsh_path_job *job) {
    if (!job) return;
    job->cancel.store(1);
    // only renders still running are told (see mtsh_path_job::sent)
    for (size_t g = 0; g < job->handles.size(); ++g) {
        std::lock_guard<std::mutex> gl(job->gpuLock[g]);
        if (job->rendering[g]) {
            mtsg_cancel(job->handles[g]);
            job->sent[g] = 1;
        }
    }
}

void mtsh_path_job_destroy(mtsh_path_job *job) {
    if (!job) return;
    for (auto *h : job->handles) mtsg_scene_destroy(h);
    delete job;
}

int mtsh_path_render(const mtsh_scene *scene, const mtsg_render_params *params, int n_gpus, float *rgbaw_out,
                     double *seconds_out) {
    mtsh_path_job *job = nullptr;
    int rc = mtsh_path_job_create(scene, n_gpus, &job);
    if (rc != MTSG_OK) return rc;
    rc = mtsh_path_job_render(job, params, rgbaw_out, seconds_out);
    mtsh_path_job_destroy(job);
    return rc;
}

void mtsh_path_last_error(char *buf, size_t size) {
    if (!buf || !size) return;
    strncpy(buf, g_perr.c_str(), size - 1);
    buf[size - 1] = 0;
}

}  // extern "C"
