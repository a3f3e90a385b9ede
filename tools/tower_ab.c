/* tower_ab.c -- A/B timing of kernel variants of libaz.so (python-free).
 * Each argument after the weights file is a path to a libaz.so build (e.g. one per -D knob,
 * `make -C alphazero-chess_amd/csrc OUT=... OBJDIR=... EXTRA=-D...`).  For every library, in
 * ROUNDS interleaved passes (DVFS drift cancels): self-play 2048 games x S sims x 1 move with the
 * 20x256 net and report the engine's own HIP-event tower time per simulation step.
 * Usage: tools/tower_ab games sims blocks filters w.f32 lib1.so [lib2.so ...] */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/az.h"

typedef struct {
    void* h;
    const char* path;
    const char* (*last_error)(void);
    int (*net_create)(const az_net_desc*, const float*, size_t, int, az_net**);
    int (*net_destroy)(az_net*);
    int (*default_cfg)(az_search_cfg*);
    int (*search_create)(az_net*, const az_search_cfg*, int, az_search**);
    int (*search_destroy)(az_search*);
    int (*reset)(az_search*);
    int (*step)(az_search*, int*, int*);
    int (*timing)(az_search*, az_timing*, int, int);
    int (*sync)(int);
} lib_t;

#define SYM(L, f, n) do { *(void**)&L->f = dlsym(L->h, n); if (!L->f) { fprintf(stderr, "%s: no %s\n", L->path, n); exit(1); } } while (0)
#define CHECK(L, x) do { if ((x) != 0) { fprintf(stderr, "%s: %s: %s\n", L->path, #x, L->last_error()); exit(1); } } while (0)

static void open_lib(lib_t* L, const char* path) {
    L->path = path;
    L->h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!L->h) { fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); exit(1); }
    SYM(L, last_error, "az_last_error");
    SYM(L, net_create, "az_net_create");
    SYM(L, net_destroy, "az_net_destroy");
    SYM(L, default_cfg, "az_search_default_cfg");
    SYM(L, search_create, "az_search_create");
    SYM(L, search_destroy, "az_search_destroy");
    SYM(L, reset, "az_selfplay_reset");
    SYM(L, step, "az_selfplay_step");
    SYM(L, timing, "az_search_timing");
    SYM(L, sync, "az_device_synchronize");
}

int main(int argc, char** argv) {
    if (argc < 7) { fprintf(stderr, "usage: tower_ab games sims blocks filters w.f32 lib.so...\n"); return 2; }
    const int games = atoi(argv[1]), sims = atoi(argv[2]), blocks = atoi(argv[3]), filters = atoi(argv[4]);
    const int nlib = argc - 6;
    lib_t* libs = calloc(nlib, sizeof(lib_t));
    for (int i = 0; i < nlib; i++) open_lib(&libs[i], argv[6 + i]);
    size_t n = (size_t)0;
    {
        size_t (*np)(int, int) = (size_t(*)(int, int))dlsym(libs[0].h, "az_net_num_params");
        n = np(blocks, filters);
    }
    float* w = malloc(n * sizeof(float));
    FILE* f = fopen(argv[5], "rb");
    if (!f || fread(w, sizeof(float), n, f) != n) { fprintf(stderr, "cannot read weights\n"); return 1; }
    fclose(f);
    const int ROUNDS = 3;
    double* best = calloc(nlib, sizeof(double));
    for (int r = 0; r < ROUNDS; r++) {
        for (int i = 0; i < nlib; i++) {
            lib_t* L = &libs[i];
            const char* dt = getenv("DTYPE");
            az_net_desc d = {blocks, filters, dt && dt[0] == 'b' ? AZ_DTYPE_BF16 : AZ_DTYPE_F32};
            az_net* net;
            CHECK(L, L->net_create(&d, w, n, 0, &net));
            az_search_cfg cfg;
            CHECK(L, L->default_cfg(&cfg));
            cfg.games = games; cfg.sims = sims; cfg.seed = 42; cfg.continuous = 1; cfg.cache_capacity = 0;
            az_search* sp;
            CHECK(L, L->search_create(net, &cfg, 0, &sp));
            CHECK(L, L->reset(sp));
            int fin = 0, act = 0;
            CHECK(L, L->step(sp, &fin, &act));             /* warm-up move */
            az_timing t;
            CHECK(L, L->timing(sp, &t, 1, 1));
            CHECK(L, L->step(sp, &fin, &act));
            CHECK(L, L->sync(0));
            CHECK(L, L->timing(sp, &t, 0, 0));
            const double ms = t.tower_ms / (double)t.sim_steps;
            const double tf = t.tower_flop / (t.tower_ms * 1e-3) / 1e12;
            /* one more move without events: wall time per move (every kernel, gaps included) */
            struct timespec t0, t1;
            CHECK(L, L->sync(0));
            clock_gettime(CLOCK_MONOTONIC, &t0);
            CHECK(L, L->step(sp, &fin, &act));
            CHECK(L, L->sync(0));
            clock_gettime(CLOCK_MONOTONIC, &t1);
            const double move_ms = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6;
            printf("round %d  %-40s tower %.4f ms/step  %.1f TFLOP/s  sim_step %.4f ms  move %.2f ms (%.0f sims/s)\n", r,
                   L->path, ms, tf, t.sim_step_ms / (double)t.sim_steps, move_ms, games * (double)sims / (move_ms * 1e-3));
            fflush(stdout);
            if (best[i] == 0 || ms < best[i]) best[i] = ms;
            L->search_destroy(sp);
            L->net_destroy(net);
        }
    }
    for (int i = 0; i < nlib; i++) printf("best %-40s %.4f ms\n", libs[i].path, best[i]);
    return 0;
}
