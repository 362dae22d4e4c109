/*
 * asan_driver.c — TEST INFRASTRUCTURE ONLY (SURVEY §5 "compile the CPU restatement with
 * -fsanitize=address,undefined"). A standalone executable linking oracle.c under AddressSanitizer
 * and UBSan (oracle/Makefile target `asan`), so the sanitizer runtime owns the process and no
 * preload is needed. It replays a scenario file written by tests/test_oracle_asan.py: a model
 * description, sim / task parameters, env origins and an action sequence; it runs
 * orc_env_step over it (resets, substeps, contacts, task math) and writes the last step's
 * obs / rew / reset / progress so the test can compare them with liboracle.so bit for bit.
 *
 * Scenario layout (little endian, no padding):
 *   int32 dyn_kind, root_free, L, G, S, P
 *   int32 parent[L], jtype[L]; f32 axis[3L], pos[3L], quat[4L], mass[L], com[3L], inertia[6L],
 *   lower[L], upper[L], damping[L], armature[L]; int32 geom_link[G], geom_type[G];
 *   f32 geom_p0[3G], geom_p1[3G], geom_radius[G]; int32 sensor_link[S]; f32 sensor_pos[3S];
 *   int32 pairs[2P]; f32 cart[6]
 *   mi_sim_params (raw struct bytes)
 *   mi_task_params (raw struct bytes; pointer fields ignored) + f32 gears[A], ratio[A], init[D]
 *   int32 N; uint64 seed; f32 origins[3N]
 *   int32 steps, substeps, A, O; f32 actions[steps * N * A]
 * Output: f32 obs[N*O], f32 rew[N], int64 reset[N], int64 progress[N].
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static FILE* g_in;

static void rd(void* dst, size_t bytes) {
    if (bytes && fread(dst, 1, bytes, g_in) != bytes) {
        fprintf(stderr, "asan_driver: truncated scenario\n");
        exit(3);
    }
}

static void* rd_new(size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) exit(4);
    rd(p, bytes);
    return p;
}

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: asan_driver <scenario.bin> <out.bin>\n");
        return 2;
    }
    g_in = fopen(argv[1], "rb");
    if (!g_in) return 2;
    int32_t hdr[6];
    rd(hdr, sizeof hdr);
    const int L = hdr[2], G = hdr[3], S = hdr[4], P = hdr[5];
    mi_model_desc m;
    memset(&m, 0, sizeof m);
    m.dyn_kind = hdr[0]; m.root_free = hdr[1]; m.num_links = L; m.num_geoms = G;
    m.num_sensors = S; m.num_pairs = P;
    m.parent = rd_new(4u * L); m.jtype = rd_new(4u * L);
    m.axis = rd_new(12u * L); m.pos = rd_new(12u * L); m.quat = rd_new(16u * L);
    m.mass = rd_new(4u * L); m.com = rd_new(12u * L); m.inertia = rd_new(24u * L);
    m.lower = rd_new(4u * L); m.upper = rd_new(4u * L); m.damping = rd_new(4u * L);
    m.armature = rd_new(4u * L);
    m.geom_link = rd_new(4u * G); m.geom_type = rd_new(4u * G);
    m.geom_p0 = rd_new(12u * G); m.geom_p1 = rd_new(12u * G); m.geom_radius = rd_new(4u * G);
    m.sensor_link = rd_new(4u * S); m.sensor_pos = rd_new(12u * S);
    m.pairs = rd_new(8u * P);
    float cart[6];
    rd(cart, sizeof cart);
    m.cart_mass = cart[0]; m.pole_mass = cart[1]; m.pole_com = cart[2];
    m.pole_inertia = cart[3]; m.cart_damping = cart[4]; m.pole_damping = cart[5];

    mi_sim_params sp;
    rd(&sp, sizeof sp);
    mi_task_params tp;
    rd(&tp, sizeof tp);
    const int A = tp.num_actions, D = L - 1;
    float* gears = rd_new(4u * A);
    float* ratio = rd_new(4u * A);
    float* init = rd_new(4u * (D > 0 ? D : 0));
    tp.joint_gears = gears; tp.motor_effort_ratio = ratio; tp.init_dof_pos = init;

    int32_t n;
    uint64_t seed;
    rd(&n, 4);
    rd(&seed, 8);
    float* origins = rd_new(12u * n);
    int32_t run[4];
    rd(run, sizeof run);
    const int steps = run[0], substeps = run[1], O = run[3];
    if (run[2] != A || O != tp.num_obs) {
        fprintf(stderr, "asan_driver: action / obs width mismatch\n");
        return 5;
    }
    float* actions = rd_new(4u * (size_t)steps * n * A);
    fclose(g_in);

    orc_set_threads(1);
    orc_sim* s = orc_sim_create(&m, &sp, n, 0, origins, seed);
    if (!s) return 6;
    orc_task_configure(s, &tp);
    float* obs = calloc((size_t)n * O, 4);
    float* obs_task = calloc((size_t)n * O, 4);
    float* rew = calloc(n, 4);
    int64_t* reset = calloc(n, 8);
    int64_t* progress = calloc(n, 8);
    float* pot = calloc(n, 4);
    float* prev = calloc(n, 4);
    float* act_out = calloc((size_t)n * (A > 0 ? A : 1), 4);
    for (int i = 0; i < n; ++i) reset[i] = 1;     /* VecEnvRLGames.reset: every env flagged */
    for (int k = 0; k < steps; ++k)
        orc_env_step(s, actions + (size_t)k * n * A, substeps, obs, obs_task, rew, reset, progress,
                     pot, prev, act_out);
    FILE* out = fopen(argv[2], "wb");
    if (!out) return 7;
    fwrite(obs, 4, (size_t)n * O, out);
    fwrite(rew, 4, n, out);
    fwrite(reset, 8, n, out);
    fwrite(progress, 8, n, out);
    fclose(out);
    orc_sim_destroy(s);
    free(obs); free(obs_task); free(rew); free(reset); free(progress); free(pot); free(prev);
    free(act_out); free(actions); free(origins); free(gears); free(ratio); free(init);
    free((void*)m.parent); free((void*)m.jtype); free((void*)m.axis); free((void*)m.pos);
    free((void*)m.quat); free((void*)m.mass); free((void*)m.com); free((void*)m.inertia);
    free((void*)m.lower); free((void*)m.upper); free((void*)m.damping); free((void*)m.armature);
    free((void*)m.geom_link); free((void*)m.geom_type); free((void*)m.geom_p0);
    free((void*)m.geom_p1); free((void*)m.geom_radius); free((void*)m.sensor_link);
    free((void*)m.sensor_pos); free((void*)m.pairs);
    return 0;
}
