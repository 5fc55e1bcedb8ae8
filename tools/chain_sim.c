// chain_sim.c — per-pixel sample-chain model of the wavefront engine with speculative
// sample starts (analysis only; input from tools/chain_log.py, driven by tools/chain_model.py).
//
// A pixel's samples run in order: sample j's RNG start state is the state sample j-1 ended
// with, and a sample with b shaded bounces takes b path steps (camera-ahead steps: the step
// that ends a sample shades the next one's camera hit). A speculative runner starts sample j
// before j-1 is done, from the state j-1 would end with if it (and every unverified sample
// before it) took `pred` bounces; it is right exactly when they all did. Runners finish in any
// order; results are taken in sample order (the fin sums), and a wrong guess discards every
// runner past the sample that broke it.
//
// Per pixel, per iteration t: runners finish, the frontier v takes finished samples in order,
// a broken guess kills the runners past v, then the window refills up to K runners (K_lo
// before iteration t_spec, K_hi from it). Output: hist[t] = runners stepping at t, summed over
// pixels; per-pixel finish iteration; total runner steps (work).
//
//   gcc -O2 -shared -fPIC tools/chain_sim.c -o /tmp/libchain_sim.so
#include <stdint.h>
#include <string.h>

#define MAXK 64

// pred_mode: 0 = constant `pred`; 1 = the pixel's last verified sample's b (pred before any)
long chain_sim(const uint16_t* b_all, int n_px, int spp, int k_lo, int k_hi, int t_spec, int pred, int pred_mode,
               int32_t* hist, int hist_len, int32_t* finish, int64_t* work_out)
{
    int64_t work = 0;
    long t_max = 0;
    for (int p = 0; p < n_px; p++) {
        const uint16_t* b = b_all + (size_t)p * spp;
        int rj[MAXK], rend[MAXK], rok[MAXK], nr = 0;  // active runners: sample, finish time, right start
        // done[j]: finished result waiting for the frontier (1 right, 2 wrong)
        static uint8_t done[1 << 16];
        memset(done, 0, spp);
        int v = 0, next = 0, t = 0, last_b = pred;
        for (;;) {
            // refill (at t, after finishes/verification of the previous iteration)
            const int K = t < t_spec ? k_lo : k_hi;
            const int pr = pred_mode == 1 ? last_b : pred;
            while (nr < K && next < spp) {
                int ok = 1;
                for (int k = v; k < next; k++)
                    if (b[k] != pr) { ok = 0; break; }
                // a wrong start runs a sample of some other length (a proxy from the same pixel)
                const int len = ok ? b[next] : b[(next * 7 + 13) % spp];
                rj[nr] = next;
                rend[nr] = t + (len > 0 ? len : 1);
                rok[nr] = ok;
                nr++;
                next++;
            }
            if (t < hist_len) hist[t] += nr;
            work += nr;
            t++;
            // finishes at t
            for (int i = 0; i < nr;)
                if (rend[i] <= t) {
                    done[rj[i]] = rok[i] ? 1 : 2;
                    rj[i] = rj[nr - 1], rend[i] = rend[nr - 1], rok[i] = rok[nr - 1];
                    nr--;
                } else
                    i++;
            // the frontier takes finished right samples in order
            while (v < spp && done[v] == 1) {
                const int bv = b[v];
                const int pr_used = pred_mode == 1 ? last_b : pred;
                last_b = bv;
                v++;
                if (bv != pr_used) {  // every runner / result past v assumed otherwise
                    for (int k = v; k < next; k++) done[k] = 0;
                    nr = 0;
                    next = v;
                    break;
                }
            }
            if (v < spp && done[v] == 2) {  // (cannot happen: the frontier's runner starts right)
                done[v] = 0;
                nr = 0;
                next = v;
            }
            if (v >= spp) break;
        }
        finish[p] = t;
        if (t > t_max) t_max = t;
    }
    *work_out = work;
    return t_max;
}

// Lattice speculation. Sample m's RNG start state is the post-warm-up state advanced by
// 2m + D*B draws, B = the shaded bounces of samples 0..m-1, so every candidate start is a
// lattice cell (m, B) and cells of one pixel merge instead of multiplying: a runner on cell
// (m, B) is right iff B is the pixel's true B_m. From iteration t0 on (the frontier then at
// (m0, B_m0)), each pixel keeps up to R runners on the cells most likely to lie on its path:
// cell (m_f + j, B_f + x) with probability P(the next j samples take x bounces), from the
// pixel's bounce histogram so far (+1 prior), j < J. Before t0 a pixel runs alone (K = 1).
// Returns the pixel's finish iteration; hist / work as chain_sim.
#define LJ 16
#define LX (8 * LJ + 1)
long lattice_sim(const uint16_t* b_all, int n_px, int spp, int R, int t0, int J, int32_t* hist, int hist_len,
                 int32_t* finish, int64_t* work_out)
{
    int64_t work = 0;
    long t_max = 0;
    static int Btrue[1 << 16 + 1];
    static uint8_t st[1 << 12][LX];  // cells (m - m_f, x): 0 none, 1 running, 2 done
    static int cend[1 << 12][LX];
    if (J > LJ) J = LJ;
    for (int p = 0; p < n_px; p++) {
        const uint16_t* b = b_all + (size_t)p * spp;
        Btrue[0] = 0;
        for (int m = 0; m < spp; m++) Btrue[m + 1] = Btrue[m] + b[m];
        // K = 1 until t0: the frontier after t0 steps
        int m_f = 0, t = 0;
        while (m_f < spp && t + b[m_f] <= t0) {
            for (int k = 0; k < b[m_f]; k++)
                if (t + k < hist_len) hist[t + k] += 1;
            work += b[m_f];
            t += b[m_f];
            m_f++;
        }
        if (m_f >= spp) {
            finish[p] = t;
            if (t > t_max) t_max = t;
            continue;
        }
        double h[9] = {0};
        for (int k = 1; k <= 8; k++) h[k] = 1.0;
        for (int m = 0; m < m_f; m++) h[b[m]] += 1.0;
        memset(st, 0, sizeof(st[0]) * (size_t)(J + 1));
        int running = 0;
        // (cells are indexed relative to the frontier; they shift when it moves)
        int cand_j[LJ * LX], cand_x[LJ * LX], nc = 0;
        int dirty = 1;
        // a sample already in progress at t0 continues on its runner
        st[0][0] = 1;
        cend[0][0] = t + b[m_f];
        running = 1;
        unsigned rs = 12345u + p;
        for (;;) {
            if (dirty) {  // candidate order for this frontier
                double pr[LJ][LX];
                memset(pr, 0, sizeof(pr));
                pr[0][0] = 1.0;
                double tot = 0;
                for (int k = 1; k <= 8; k++) tot += h[k];
                for (int j = 1; j < J; j++)
                    for (int x = 0; x < LX; x++)
                        if (pr[j - 1][x] > 0)
                            for (int k = 1; k <= 8 && x + k < LX; k++) pr[j][x + k] += pr[j - 1][x] * h[k] / tot;
                nc = 0;
                for (int j = 0; j < J && m_f + j < spp; j++)
                    for (int x = 0; x < LX; x++)
                        if (pr[j][x] > 1e-4) cand_j[nc] = j, cand_x[nc] = x, nc++;
                // sort by probability (insertion; nc is small)
                for (int i = 1; i < nc; i++) {
                    int jj = cand_j[i], xx = cand_x[i], k = i - 1;
                    double v = pr[jj][xx];
                    while (k >= 0 && pr[cand_j[k]][cand_x[k]] < v) {
                        cand_j[k + 1] = cand_j[k], cand_x[k + 1] = cand_x[k];
                        k--;
                    }
                    cand_j[k + 1] = jj, cand_x[k + 1] = xx;
                }
                dirty = 0;
            }
            for (int i = 0; i < nc && running < R; i++) {
                const int j = cand_j[i], x = cand_x[i];
                if (st[j][x]) continue;
                const int m = m_f + j;
                const int right = Btrue[m] - Btrue[m_f] == x;
                int len = right ? b[m] : 0;
                if (!right) {  // some sample of the pixel's distribution
                    rs = rs * 1103515245u + 12345u;
                    len = b[(rs >> 8) % (unsigned)spp];
                }
                st[j][x] = 1;
                cend[j][x] = t + len;
                running++;
            }
            if (t < hist_len) hist[t] += running;
            work += running;
            t++;
            for (int j = 0; j < J; j++)
                for (int x = 0; x < LX; x++)
                    if (st[j][x] == 1 && cend[j][x] <= t) st[j][x] = 2, running--;
            // the frontier walks done cells of the true path
            int moved = 0;
            while (m_f < spp && st[0][0] == 2) {
                const int bb = b[m_f];
                h[bb] += 1.0;
                m_f++;
                moved = 1;
                // shift cells: new (j, x) = old (j + 1, x + bb)
                for (int j = 0; j < J; j++)
                    for (int x = 0; x < LX; x++) {
                        const int oj = j + 1, ox = x + bb;
                        if (oj < J && ox < LX) {
                            st[j][x] = st[oj][ox];
                            cend[j][x] = cend[oj][ox];
                        } else
                            st[j][x] = 0;
                    }
            }
            if (moved) {  // runners on dropped cells stop
                running = 0;
                for (int j = 0; j < J; j++)
                    for (int x = 0; x < LX; x++) running += st[j][x] == 1;
                dirty = 1;
            }
            if (m_f >= spp) break;
        }
        finish[p] = t;
        if (t > t_max) t_max = t;
    }
    *work_out = work;
    return t_max;
}
