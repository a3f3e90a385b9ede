/* tower_trace.c -- phase stamps of the f32 Winograd tower (an AZ_TOWER_TRACE build of libaz.so,
 * tools/build_variants.sh trace=-DAZ_TOWER_TRACE).  Self-play of G games x S sims x 2 moves with
 * the B x F net, then the stamps of the last tower launch (8 workgroups x 8 waves) go to out.bin;
 * tools/tower_trace.py summarises them.
 * Usage: tools/tower_trace games sims blocks filters w.f32 lib.so out.bin */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/az.h"

#define SYM(f, n) do { *(void**)&f = dlsym(h, n); if (!f) { fprintf(stderr, "no %s\n", n); return 1; } } while (0)
#define CHECK(x) do { if ((x) != 0) { fprintf(stderr, "%s: %s\n", #x, last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    if (argc < 8) { fprintf(stderr, "usage: tower_trace games sims blocks filters w.f32 lib.so out.bin\n"); return 2; }
    const int games = atoi(argv[1]), sims = atoi(argv[2]), blocks = atoi(argv[3]), filters = atoi(argv[4]);
    void* h = dlopen(argv[6], RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 1; }
    const char* (*last_error)(void);
    size_t (*num_params)(int, int);
    int (*net_create)(const az_net_desc*, const float*, size_t, int, az_net**);
    int (*default_cfg)(az_search_cfg*);
    int (*search_create)(az_net*, const az_search_cfg*, int, az_search**);
    int (*reset)(az_search*);
    int (*step)(az_search*, int*, int*);
    int (*trace_read)(unsigned long long*, size_t);
    SYM(last_error, "az_last_error"); SYM(num_params, "az_net_num_params"); SYM(net_create, "az_net_create");
    SYM(default_cfg, "az_search_default_cfg"); SYM(search_create, "az_search_create");
    SYM(reset, "az_selfplay_reset"); SYM(step, "az_selfplay_step"); SYM(trace_read, "az_tower_trace_read");
    const size_t n = num_params(blocks, filters);
    float* w = malloc(n * sizeof(float));
    FILE* f = fopen(argv[5], "rb");
    if (!f || fread(w, sizeof(float), n, f) != n) { fprintf(stderr, "cannot read weights\n"); return 1; }
    fclose(f);
    az_net_desc d = {blocks, filters, AZ_DTYPE_F32};
    az_net* net;
    CHECK(net_create(&d, w, n, 0, &net));
    az_search_cfg cfg;
    CHECK(default_cfg(&cfg));
    cfg.games = games; cfg.sims = sims; cfg.seed = 42; cfg.continuous = 1; cfg.cache_capacity = 0;
    az_search* sp;
    CHECK(search_create(net, &cfg, 0, &sp));
    CHECK(reset(sp));
    int fin = 0, act = 0;
    CHECK(step(sp, &fin, &act));
    CHECK(step(sp, &fin, &act));
    const size_t cnt = 8 * 8 * 2048;
    unsigned long long* t = calloc(cnt, 8);
    if (trace_read(t, cnt) != 0) { fprintf(stderr, "trace read failed\n"); return 1; }
    FILE* o = fopen(argv[7], "wb");
    if (!o || fwrite(t, 8, cnt, o) != cnt) { fprintf(stderr, "cannot write %s\n", argv[7]); return 1; }
    fclose(o);
    printf("tower_trace: %d games x %d sims, %dx%d: stamps of the last launch in %s\n", games, sims, blocks, filters, argv[7]);
    return 0;
}
