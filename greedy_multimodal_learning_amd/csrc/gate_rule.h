// The on-device conditional-learning-speed gate's step rule (Bias_Mitigation_Strong.on_backward_end,
// reference src/callbacks.py:199-267) as device functions of one thread: k_gate_strong /
// k_gate_strong_n (gate.hip) and the group-sum finalize that runs the rule in its own launch
// (k_group_finalize, group_sumsq.hip: gm_group_sumsq_gate).  s: the step's group sums (fp64).
#pragma once
#include "gm_common.h"

namespace gm {

__device__ inline void gate_strong_rule(const double* s, gm_gate_state* st) {
    gm_gate_state g = *st;
    if (g.curation_mode) ++g.n_curated;  // the step that just ran was curated
    auto bdr = [&]() {
        // s = [w_main0, g_main0, w_main1, g_main1, w_by0, g_by0, w_by1, g_by1]
        g.M[2] += s[1] / s[0];
        g.M[3] += s[3] / s[2];
        g.M[0] += s[5] / s[4];
        g.M[1] += s[7] / s[6];
        g.d_bdr = log10(g.M[0] / g.M[2]) - log10(g.M[1] / g.M[3]);
    };
    if (g.unlock) {
        if (!g.curation_mode) {
            bdr();
            if (fabs(g.d_bdr) > g.eps) {
                g.curation_mode = 1;
                g.curation_step = 0;
                g.caring = g.d_bdr < 0.0 ? 1 : 0;
            } else {
                g.curation_mode = 0;
                g.caring = 0;
            }
        } else {
            g.curation_step += 1;
            if (g.curation_step == g.window) g.curation_mode = 0;
        }
    } else {
        bdr();
        g.curation_mode = 0;
        g.caring = 0;
    }
    *st = g;
}

// N branches (C4 / C5): the host gate's N-branch rule (callbacks.bdr_values /
// bdr_decision) in fp64 - M_main_i += g/w of group i, M_bypass_i += g/w of group nb+i,
// BDR_i = log10(M_bypass_i / M_main_i), d = max - min (two branches: the signed
// BDR_0 - BDR_1), caring = argmax (first on ties)
__device__ inline void gate_strong_rule_n(const double* s, gm_gate_state_n* st) {
    gm_gate_state_n g = *st;
    const int nb = g.nb < 0 ? 0 : (g.nb > GM_GATE_MAX_BRANCHES ? GM_GATE_MAX_BRANCHES : g.nb);
    if (g.curation_mode) ++g.n_curated;
    int hi = 0;
    auto bdr = [&]() {
        double mx = 0.0, mn = 0.0;
        for (int i = 0; i < nb; ++i) {
            g.M_main[i] += s[2 * i + 1] / s[2 * i];
            g.M_bypass[i] += s[2 * (nb + i) + 1] / s[2 * (nb + i)];
            const double b = log10(g.M_bypass[i] / g.M_main[i]);
            g.bdr[i] = b;
            if (i == 0 || b > mx) { mx = b; hi = i; }  // numpy argmax: first maximum
            if (i == 0 || b < mn) mn = b;
        }
        // two branches: the reference's signed BDR_0 - BDR_1 (src/callbacks.py:233), as the
        // host gate and k_gate_strong log it; the decision (|d| > eps, caring = argmax) is the same
        g.d_bdr = nb == 2 ? g.bdr[0] - g.bdr[1] : mx - mn;
    };
    if (g.unlock) {
        if (!g.curation_mode) {
            bdr();
            if (fabs(g.d_bdr) > g.eps) {
                g.curation_mode = 1;
                g.curation_step = 0;
                g.caring = hi;
            } else {
                g.curation_mode = 0;
                g.caring = 0;
            }
        } else {
            g.curation_step += 1;
            if (g.curation_step == g.window) g.curation_mode = 0;
        }
    } else {
        bdr();
        g.curation_mode = 0;
        g.caring = 0;
    }
    *st = g;
}

}  // namespace gm
