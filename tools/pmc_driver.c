/* pmc_driver.c -- a python-free driver for rocprofv3 PMC passes: self-play through the C-ABI
 * (include/az.h) with the 20x256 net (random weights, Kaiming-uniform bounds as in
 * azchess.random_weights), G games, S sims, one move.  Each simulation step launches the fused
 * tower in search mode once, exactly as bench.py's timed region does.
 * Weights: the flat f32 layout of az_net_num_params, written by
 *   python3 -c "import azchess as A; A.random_weights(20, 256, seed=42).tofile('w.f32')"
 * Build: make -C tools   Run: tools/pmc_driver games sims moves blocks filters w.f32 [f32|bf16] */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../include/az.h"

#define CHECK(x) do { if ((x) != 0) { fprintf(stderr, "%s: %s\n", #x, az_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    if (argc < 7) { fprintf(stderr, "usage: pmc_driver games sims moves blocks filters weights.f32\n"); return 2; }
    int games = atoi(argv[1]), sims = atoi(argv[2]), moves = atoi(argv[3]);
    int blocks = atoi(argv[4]), filters = atoi(argv[5]);
    size_t n = az_net_num_params(blocks, filters);
    float* w = (float*)malloc(n * sizeof(float));
    FILE* f = fopen(argv[6], "rb");
    if (!f || fread(w, sizeof(float), n, f) != n) { fprintf(stderr, "cannot read %zu weights from %s\n", n, argv[6]); return 1; }
    fclose(f);
    const int bf = argc > 7 && argv[7][0] == 'b';
    az_net_desc d = {blocks, filters, bf ? AZ_DTYPE_BF16 : AZ_DTYPE_F32};
    az_net* net;
    CHECK(az_net_create(&d, w, n, 0, &net));
    az_search_cfg cfg;
    CHECK(az_search_default_cfg(&cfg));
    cfg.games = games; cfg.sims = sims; cfg.seed = 42; cfg.continuous = 1; cfg.cache_capacity = 0;
    az_search* sp;
    CHECK(az_search_create(net, &cfg, 0, &sp));
    CHECK(az_selfplay_reset(sp));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int fin = 0, act = 0;
    for (int m = 0; m < moves; m++) CHECK(az_selfplay_step(sp, &fin, &act));
    CHECK(az_device_synchronize(0));
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double dt = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    printf("pmc_driver: %d games x %d sims x %d moves, %dx%d %s: %.3f s (%.0f sims/s)\n", games, sims, moves, blocks,
           filters, bf ? "bf16" : "f32", dt, (double)games * sims * moves / dt);
    az_search_destroy(sp);
    az_net_destroy(net);
    free(w);
    return 0;
}
