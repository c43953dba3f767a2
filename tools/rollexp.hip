// Rollout variants side by side: each variant steps its own env (same seed) through the same
// launches, the results are compared byte for byte with variant 0 (boards, meta, episode
// counters, clocks, every ring section), then each is timed over graph-replayed launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rollexp.hip -o tools/rollexp
//   tools/rollexp [n=65536] [K=64]
#include "../reinforcement-learning-2048_amd/csrc/g2048.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

void launch_old(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout<true, true, false>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

void launch_lean(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_lean<false, false, true>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

template <int kStores>
void launch_part(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_lean<false, false, true, kStores>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

// The ring stores alone (no board arithmetic): the rollout's store pattern with a cheap per-step
// value, to price the store stream at large N.  kAux: the buffer stores' cache-policy bits
// (2 = nt).
template <int kStores, int kAux>
__global__ __launch_bounds__(kBlock) void k_store_only(StepArgs A) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= A.n) return;
    const uint32_t n32 = (uint32_t)A.n, cap32 = (uint32_t)A.rb.capacity, lane = (uint32_t)i;
    const uint64_t t0 = load_clock(A.clock, i);
    uint32_t soff = (uint32_t)ring_row(t0, A.rb.rows) * n32;
    __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(A.rb.win, 0, (int)A.rb.win_bytes, 0x00020000);
    const uint32_t v_s = A.rb.o_s + 16u * lane, v_s2 = A.rb.o_s2 + 16u * lane;
    const uint32_t v_a = A.rb.o_a + lane, v_r = A.rb.o_r + 4u * lane, v_d = A.rb.o_d + lane;
    uint32_t x = lane * 2654435761u;
    for (int s = 0; s < A.k_steps; ++s) {
        x = x * 1664525u + 1013904223u;
        if constexpr (kStores & 1)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{x, x + 1u, x + 2u, x + 3u}, rw, v_s, soff * 16u, kAux);
        if constexpr ((kStores & 2) != 0)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{x ^ 1u, x ^ 2u, x ^ 3u, x}, rw, v_s2, soff * 16u, kAux);
        if constexpr ((kStores & 4) != 0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)x, rw, v_a, soff, kAux);
        if constexpr ((kStores & 8) != 0) __builtin_amdgcn_raw_buffer_store_b32(x, rw, v_r, soff * 4u, kAux);
        if constexpr ((kStores & 16) != 0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(x >> 8), rw, v_d, soff, kAux);
        soff = soff + n32 == cap32 ? 0u : soff + n32;
    }
}

// A warp-specialised large-N rollout, measured and not kept: workgroups of 512
// threads.  Past ~256k boards the ring streams to HBM and the launch is
// store-bound, and in k_rollout_lean every wave both computes and stores: with the store queue
// full, all waves of a SIMD end up waiting at their stores together, so compute and stores
// barely overlap (4M boards x 16: 261 us of compute + 480 us of stores -> 700-745 us).  Here
// waves 0-3 step the workgroup's 256 boards and write each transition into an LDS double
// buffer; waves 4-7 copy the previous step's buffer to the ring.  One barrier per step, so a
// step would cost max(compute, store issue) instead of their sum -- but it measured the sum all
// the same (4M x 16: 738 us).  Bitwise the same transitions as k_rollout_lean.
struct WsBuf {
    uint4 s[kBlock];
    uint4 s2[kBlock];
    uint32_t r[kBlock];
    uint8_t a[kBlock];
    uint8_t d[kBlock];
};

template <bool kSum, bool kP410>
__global__ __launch_bounds__(2 * kBlock) void k_rollout_ws_barrier(StepArgs A) {
    __shared__ uint4 s_dir[8];
    __shared__ WsBuf buf[2];
    const bool storer = threadIdx.x >= kBlock;
    const int j = storer ? (int)threadIdx.x - kBlock : (int)threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * kBlock + j;
    const bool live = i < A.n;
    uint64_t c0 = 0;
    if (live) c0 = A.clock[i >> 6];
    if (threadIdx.x < 8) s_dir[threadIdx.x] = reinterpret_cast<const uint4*>(&kDirNet[0][0][0])[threadIdx.x];
    const uint64_t t0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)c0) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(c0 >> 32)) << 32);
    const int K = A.k_steps > 0 ? A.k_steps : 0;
    __syncthreads();
    if (storer) {
        // the ring side: step s's transition of board i from buf[s & 1] to ring row (t0 + s) mod rows
        const uint32_t cap32 = (uint32_t)A.rb.capacity, n32 = (uint32_t)A.n;
        uint32_t soff = (uint32_t)ring_row(t0, A.rb.rows) * n32;
        __amdgpu_buffer_rsrc_t rw =
            __builtin_amdgcn_make_buffer_rsrc(A.rb.win, 0, (int)A.rb.win_bytes, 0x00020000);
        const uint32_t lane = (uint32_t)i;
        const uint32_t v_s = A.rb.o_s + 16u * lane, v_s2 = A.rb.o_s2 + 16u * lane;
        const uint32_t v_a = A.rb.o_a + lane, v_r = A.rb.o_r + 4u * lane, v_d = A.rb.o_d + lane;
        for (int s = 0; s < K; ++s) {
            __syncthreads();  // buf[s & 1] holds step s
            const WsBuf& B = buf[s & 1];
            if (live) {
                const uint4 sv = B.s[j], s2v = B.s2[j];
                const uint32_t rv = B.r[j];
                const uint8_t av = B.a[j], dv = B.d[j];
                store_board(Board{sv.x, sv.y, sv.z, sv.w}, rw, v_s, soff * 16u);
                store_board(Board{s2v.x, s2v.y, s2v.z, s2v.w}, rw, v_s2, soff * 16u);
                __builtin_amdgcn_raw_buffer_store_b8(av, rw, v_a, soff, 0);
                __builtin_amdgcn_raw_buffer_store_b32(rv, rw, v_r, soff * 4u, 0);
                __builtin_amdgcn_raw_buffer_store_b8(dv, rw, v_d, soff, 0);
            }
            soff = soff + n32 == cap32 ? 0u : soff + n32;
        }
        return;
    }
    // the board side
    Board b{0u, 0u, 0u, 0u};
    uint2 m = make_uint2(0, 0);
    uint4 ep = make_uint4(0, 0, 0, 0);
    if (live) {
        b = load_board(A.board[i]);
        m = load_meta(A, i, t0);
        ep = A.ep[i];
    }
    const uint64_t gid = A.board_offset + (uint64_t)i;
    const uint32_t p4 = A.p4_thresh;
    long long rsum = 0;
    const uint32_t ep0 = ep.x;
    Board last = b;
    const uint32_t k255 = opaque_255();
    uint4 blk = make_uint4(0, 0, 0, 0), vb = blk, vb2 = blk;
    for (int s = 0; s < K; ++s) {
        const uint64_t t = t0 + (uint64_t)s;
        if (s == 0 || (t & 3u) == 0u) {
            blk = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_RANDOM, t >> 2);
            value_blocks<kP410>(A.seed_lo, A.seed_hi, gid, t >> 2, vb, vb2);
        }
        const uint32_t k = (uint32_t)t & 3u;
        const uint32_t w = word_of(blk, k), v = word_of(vb, k), v2 = word_of(vb2, k);
        const uint32_t a2 = (w >> 30) * 2u;
        WsBuf& B = buf[s & 1];
        B.s[j] = make_uint4(b.r0, b.r1, b.r2, b.r3);
        bool done;
        const uint32_t r = lean_step(b, w, spawn_exp<kP410>(w, v, p4), s_dir[a2], s_dir[a2 + 1u], done, k255);
        m.x += r;
        m.y += 1u;
        if constexpr (kSum) rsum += r;
        B.s2[j] = make_uint4(b.r0, b.r1, b.r2, b.r3);
        B.a[j] = (uint8_t)(w >> 30);
        B.r[j] = r;
        B.d[j] = (uint8_t)done;
        const uint64_t dl = __builtin_amdgcn_ballot_w64(done);
        if (dl != 0u) {
            const Board f = fresh_board_w<kP410>(w, v, v2, p4);
            last.r0 = sel_lanes(dl, b.r0, last.r0);
            last.r1 = sel_lanes(dl, b.r1, last.r1);
            last.r2 = sel_lanes(dl, b.r2, last.r2);
            last.r3 = sel_lanes(dl, b.r3, last.r3);
            ep.x = sel_lanes(dl, ep.x + 1u, ep.x);
            ep.y = sel_lanes(dl, m.x, ep.y);
            ep.z = sel_lanes(dl, m.y, ep.z);
            b.r0 = sel_lanes(dl, f.r0, b.r0);
            b.r1 = sel_lanes(dl, f.r1, b.r1);
            b.r2 = sel_lanes(dl, f.r2, b.r2);
            b.r3 = sel_lanes(dl, f.r3, b.r3);
            m.x = sel_lanes(dl, 0u, m.x);
            m.y = sel_lanes(dl, 0u, m.y);
        }
        __syncthreads();  // step s is in buf[s & 1]; the ring side copies it during step s + 1
    }
    if (!live) return;
    const uint64_t t1 = t0 + (uint64_t)K;
    A.board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    store_meta(A, i, t1, m, ep.x != ep0);
    if (ep.x != ep0) {
        ep.w = max_exp(last);
        A.ep[i] = ep;
        if (A.qsum) A.qsum[i] = 0.0;
    }
    if ((i & 63) == 0) A.clock[i >> 6] = t1;
    if constexpr (kSum) A.reward_sum[i] += rsum;
    if (i == 0) bump_count(A, t1);
}

template <int kAux>
void launch_lean_aux(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_lean<false, false, true, 0x1F, 4, kAux>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

template <int kD, int kAux>
void launch_ws2(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_ws<false, false, kD, kAux>), dim3(grid_for(e->n)), dim3(2 * kBlock), 0, st, A);
}

void launch_ws(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_ws_barrier<false, false>), dim3(grid_for(e->n)), dim3(2 * kBlock), 0, st, A);
}

template <bool kQR, int kWaves>
void launch_occ(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_lean<false, false, kQR, 0x1F, kWaves>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

template <int kStores, int kAux>
void launch_store(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_store_only<kStores, kAux>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

struct Variant {
    const char* name;
    void (*fn)(g2048_env*, g2048_replay*, int, hipStream_t);
};

const Variant kVariants[] = {
    {"k_rollout (general path)", launch_old},
    {"k_rollout_lean", launch_lean},
    {"warp-specialised, barrier per step", launch_ws},
    {"lean, 5 waves/SIMD", launch_occ<true, 5>},
    {"lean no-QR, 4 waves/SIMD", launch_occ<false, 4>},
    {"lean, nt stores", launch_lean_aux<2>},
    {"lean, aux 1 (glc)", launch_lean_aux<1>},
    {"lean, aux 16 (sc1)", launch_lean_aux<16>},
    {"lean, aux 17 (sc0 sc1)", launch_lean_aux<17>},
    {"lean, aux 3 (sc0 nt)", launch_lean_aux<3>},
    {"ws, aux 1", launch_ws2<8, 1>},
    {"ws, aux 3", launch_ws2<8, 3>},
    {"ws, aux 16 (sc1)", launch_ws2<8, 16>},
    {"ws, aux 18 (sc1 nt)", launch_ws2<8, 18>},
    {"ws, aux 19 (sc0 sc1 nt)", launch_ws2<8, 19>},
    {"ws2: pair ring 4 steps", launch_ws2<4, 0>},
    {"ws2: pair ring 8 steps", launch_ws2<8, 0>},
    {"ws2: pair ring 8 steps, nt", launch_ws2<8, 2>},
    {"ws2: pair ring 12 steps, nt", launch_ws2<12, 2>},
    // timing only (parity MISMATCH expected: sections left unwritten)
    {"lean, no byte stores (a, d)", launch_part<0x0B>},
    {"lean, s + s2 only", launch_part<0x03>},
    {"lean, no ring stores", launch_part<0x00>},
    {"stores only (all five)", launch_store<0x1F, 0>},
    {"stores only (s + s2)", launch_store<0x03, 0>},
    {"stores only (all five, nt)", launch_store<0x1F, 2>},
    {"stores only (all five, sc1)", launch_store<0x1F, 16>},
    {"lean, no ring stores (sc1 build)", launch_part<0x00>},
};
constexpr int kParityVariants = 19;  // the others skip sections of the ring

template <typename T>
std::vector<T> fetch(const T* d, size_t n) {
    std::vector<T> h(n);
    (void)hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost);
    return h;
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
    const int K = argc > 2 ? atoi(argv[2]) : 64;
    const int nv = (int)(sizeof(kVariants) / sizeof(kVariants[0]));
    hipStream_t st;
    (void)hipStreamCreate(&st);
    std::vector<g2048_env*> envs(nv);
    std::vector<g2048_replay*> rbs(nv);
    for (int v = 0; v < nv; ++v) {
        if (g2048_env_create(&envs[v], n, 7, 0, 0, 0, nullptr) ||
            g2048_replay_create(&rbs[v], n * K, 0, nullptr)) {
            printf("create failed: %s\n", g2048_last_error());
            return 1;
        }
    }
    {
        StepArgs A;
        make_args(envs[0], rbs[0], A);
        if (!A.rb.win_bytes) {  // the buffer-store kernels need the ring in one < 4 GiB window
            printf("ring of %lld rows exceeds the 4 GiB buffer window: not timed\n", (long long)(n * K));
            return 1;
        }
    }
    // parity: 5 launches from the same start (an odd K first moves every clock to an odd step);
    // ROLLEXP_PHASE0=1 skips them (timing then starts from step 0, as bench.py's legs do)
    const bool phase0 = getenv("ROLLEXP_PHASE0") != nullptr;
    for (int v = 0; v < nv && !phase0; ++v) {
        kVariants[v].fn(envs[v], rbs[v], 3, st);
        for (int it = 0; it < 4; ++it) kVariants[v].fn(envs[v], rbs[v], K, st);
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    const size_t C = (size_t)n * K;
    auto b0 = fetch(envs[0]->board, n * 16);
    auto m0 = fetch(envs[0]->meta, n * 2);
    auto e0 = fetch(envs[0]->ep, n * 4);
    auto c0 = fetch(envs[0]->clock, (n + 63) / 64);
    auto s0 = fetch(rbs[0]->s, C * 16);
    auto t0 = fetch(rbs[0]->s2, C * 16);
    auto a0 = fetch(rbs[0]->a, C);
    auto r0 = fetch(rbs[0]->r, C);
    auto d0 = fetch(rbs[0]->d, C);
    int bad = 0;
    for (int v = 1; v < kParityVariants && !phase0; ++v) {
        const bool ok = fetch(envs[v]->board, n * 16) == b0 && fetch(envs[v]->meta, n * 2) == m0 &&
                        fetch(envs[v]->ep, n * 4) == e0 &&
                        fetch(envs[v]->clock, (n + 63) / 64) == c0 &&
                        fetch(rbs[v]->s, C * 16) == s0 && fetch(rbs[v]->s2, C * 16) == t0 &&
                        fetch(rbs[v]->a, C) == a0 && fetch(rbs[v]->r, C) == r0 &&
                        fetch(rbs[v]->d, C) == d0;
        printf("parity %-34s %s\n", kVariants[v].name, ok ? "bitwise equal" : "MISMATCH");
        if (!ok) {  // which outputs, and the first differing index of each
            auto first = [](const auto& x, const auto& y) -> long long {
                for (size_t k = 0; k < x.size(); ++k)
                    if (x[k] != y[k]) return (long long)k;
                return -1;
            };
            printf("  board %lld meta %lld ep %lld clock %lld s %lld s2 %lld a %lld r %lld d %lld\n",
                   first(fetch(envs[v]->board, n * 16), b0), first(fetch(envs[v]->meta, n * 2), m0),
                   first(fetch(envs[v]->ep, n * 4), e0), first(fetch(envs[v]->clock, (n + 63) / 64), c0),
                   first(fetch(rbs[v]->s, C * 16), s0), first(fetch(rbs[v]->s2, C * 16), t0),
                   first(fetch(rbs[v]->a, C), a0), first(fetch(rbs[v]->r, C), r0),
                   first(fetch(rbs[v]->d, C), d0));
            const auto sv = fetch(rbs[v]->s, C * 16);
            long long k = first(sv, s0), cnt = 0;
            for (size_t q = 0; q < sv.size(); q += 16)
                cnt += memcmp(&sv[q], &s0[q], 16) != 0;
            printf("  %lld ring rows of s differ\n", cnt);
            std::vector<long long> rowhist(C / n, 0);
            for (size_t q = 0; q < sv.size(); q += 16)
                if (memcmp(&sv[q], &s0[q], 16) != 0) rowhist[(q / 16) / n]++;
            printf("  differing s per row:");
            for (size_t q = 0; q < rowhist.size(); ++q) printf(" %lld", rowhist[q]);
            printf("\n");
            const auto tv = fetch(rbs[v]->s2, C * 16);
            const auto dv = fetch(rbs[v]->d, C);
            int shown = 0;
            for (size_t q = 0; q < sv.size() && shown < 6; q += 16) {
                if (memcmp(&sv[q], &s0[q], 16) == 0) continue;
                ++shown;
                const long long slot = q / 16, row = slot / n, bi = slot % n;
                const long long prev = ((row + (long long)(C / n) - 1) % (C / n)) * n + bi;
                printf("  row %lld board %lld (wave lane %lld)\n   s ref ", row, bi, bi & 63);
                for (int c = 0; c < 16; ++c) printf("%02x", s0[slot * 16 + c]);
                printf("\n   s var ");
                for (int c = 0; c < 16; ++c) printf("%02x", sv[slot * 16 + c]);
                printf("\n   s2prv ");
                for (int c = 0; c < 16; ++c) printf("%02x", tv[prev * 16 + c]);
                printf("  d(prev) ref %d var %d; wave's d(prev) sum %d\n", (int)d0[prev], (int)dv[prev],
                       [&] { int z = 0; for (int c = 0; c < 64; ++c) z += d0[prev - (bi & 63) + c]; return z; }());
            }
            if (false) {
                const long long slot = k / 16, row = slot / n, bi = slot % n;
                const long long prev = ((row + (long long)(C / n) - 1) % (C / n)) * n + bi;
                auto hex = [](const uint8_t* p) {
                    for (int q = 0; q < 16; ++q) printf("%x", p[q]);
                };
                printf("  row %lld board %lld\n  s  (variant 0) ", row, bi);
                hex(&s0[slot * 16]);
                printf("\n  s  (variant)   ");
                hex(&sv[slot * 16]);
                printf("\n  s2 of the previous row ");
                hex(&t0[prev * 16]);
                printf("  d %d\n", (int)d0[prev]);
            }
        }
        bad += !ok;
    }
    // timing: graphs of 20 launches, each replayed once untimed, then 10 timed replays
    hipEvent_t ev0, ev1;
    (void)hipEventCreate(&ev0);
    (void)hipEventCreate(&ev1);
    for (int rep = 0; rep < 3; ++rep) {
        for (int v = 0; v < nv; ++v) {
            hipGraph_t g;
            hipGraphExec_t ge;
            (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
            for (int it = 0; it < 20; ++it) kVariants[v].fn(envs[v], rbs[v], K, st);
            (void)hipStreamEndCapture(st, &g);
            (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(ev0, st);
            for (int it = 0; it < 10; ++it) (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(ev1, st);
            (void)hipEventSynchronize(ev1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev0, ev1);
            const double us = 1e3 * ms / 200.0;
            printf("%-36s n=%-8lld K=%-4d %8.2f us/launch  %7.1f G steps/s  %6.3f of 8 TB/s\n",
                   kVariants[v].name, (long long)n, K, us, n * K / us * 1e-3,
                   38.0 * n * K / us * 1e-6 / 8.0);
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
        }
    }
    return bad ? 2 : 0;
}
