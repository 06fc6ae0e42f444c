// Update rules of the online linear learner family, shared by the gfx950 kernel
// (csrc/kernels/linear.hip) and the C++ CPU engine (csrc/host/linear_cpu.cpp).
//
// Semantics restate Hivemall's learners (reference
// apache/incubator-hivemall core/src/main/java/hivemall/{classifier,regression,optimizer}):
//   binary classifiers : PerceptronUDTF, PassiveAggressiveUDTF(PA/PA1/PA2),
//                        ConfidenceWeightedUDTF, AROWClassifierUDTF(AROW/AROWh),
//                        SoftConfideceWeightedUDTF(SCW1/SCW2), AdaGradRDAUDTF
//   regression         : LogressUDTF, PassiveAggressiveRegressionUDTF(PA1/PA2/PA1a/PA2a),
//                        AROWRegressionUDTF(AROW/AROWe/AROWe2), AdaGradUDTF, AdaDeltaUDTF
//   general            : GeneralClassifierUDTF / GeneralRegressorUDTF = loss x optimizer x
//                        regulariser x eta schedule
//   multiclass         : MulticlassOnlineClassifierUDTF family (actual vs. best-wrong label)
//
// Per-feature state is one float4 {w, s1, s2, s3}; the meaning of s1..s3 depends on the
// algorithm / optimizer (covariance, AdaGrad sum of squares, Adam moments, ...).
// Per-replica scalar state (step counter, online target variance, Eve feedback) lives in
// a float[REP_SCALARS] block.  Every rule is a pure function so the CPU engine and the
// kernel produce the same numbers.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HM_HD __host__ __device__ __forceinline__
#else
#define HM_HD static inline __attribute__((always_inline))   // as on the device: the per-feature rules must inline into the row loop
#endif

namespace hm_lin {

// ---------------------------------------------------------------- algorithm ids
enum Algo : int {
    A_PERCEPTRON = 0, A_PA = 1, A_PA1 = 2, A_PA2 = 3, A_CW = 4, A_AROW = 5, A_AROWH = 6,
    A_SCW1 = 7, A_SCW2 = 8, A_ADAGRAD_RDA = 9,
    A_LOGRESS = 10, A_PA1_REGR = 11, A_PA2_REGR = 12, A_PA1A_REGR = 13, A_PA2A_REGR = 14,
    A_AROW_REGR = 15, A_AROWE_REGR = 16, A_AROWE2_REGR = 17, A_ADAGRAD_REGR = 18,
    A_ADADELTA_REGR = 19,
    A_GENERAL = 20,
    A_KPA = 21,  // reserved (kernel expansion PA handled on the host)
};

enum Loss : int {
    L_HINGE = 0, L_LOG = 1, L_SQUARED_HINGE = 2, L_MODIFIED_HUBER = 3, L_SQUARED = 4,
    L_QUANTILE = 5, L_EPS_INSENSITIVE = 6, L_SQ_EPS_INSENSITIVE = 7, L_HUBER = 8,
};

enum Opt : int {
    O_SGD = 0, O_MOMENTUM = 1, O_NESTEROV = 2, O_ADAGRAD = 3, O_RMSPROP = 4,
    O_RMSPROP_GRAVES = 5, O_ADADELTA = 6, O_ADAM = 7, O_NADAM = 8, O_EVE = 9, O_ADAM_HD = 10,
    O_ADAGRAD_RDA = 11,
};

enum Reg : int { R_NO = 0, R_L1 = 1, R_L2 = 2, R_ELASTIC = 3, R_RDA = 4 };
enum Eta : int { E_FIXED = 0, E_SIMPLE = 1, E_INV = 2 };

// per-replica scalars
enum RepScalar : int { RS_T = 0, RS_N = 1, RS_MEAN = 2, RS_M2 = 3, RS_EVE_D = 4, RS_EVE_F = 5,
                       RS_LOSS = 6, RS_UPDATES = 7 };
#define HM_REP_SCALARS 8

struct Params {
    int algo, loss, opt, reg, eta;
    int amsgrad;
    int n_labels;            // 1 for binary / regression
    float eta0, power_t, total_steps;
    float lambda, l1_ratio;
    float c, r, phi, epsilon;
    float alpha, beta1, beta2, eps, rho, decay, beta_hd, scale;
    float quantile_tau, huber_c;
    float init_covar;
};

struct F4 { float w, s1, s2, s3; };

// ---------------------------------------------------------------- small math
HM_HD float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
HM_HD float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }
HM_HD float log1pexpf(float x) { return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x)); }

// ---------------------------------------------------------------- losses (p, y)
// classification losses take y in {-1,+1}; regression losses take the real target.
HM_HD float loss_value(int l, float p, float y, const Params& P) {
    switch (l) {
        case L_HINGE: { float z = 1.f - y * p; return z > 0.f ? z : 0.f; }
        case L_LOG: return log1pexpf(-y * p);
        case L_SQUARED_HINGE: { float z = 1.f - y * p; return z > 0.f ? z * z : 0.f; }
        case L_MODIFIED_HUBER: {
            float z = y * p;
            if (z >= 1.f) return 0.f;
            if (z >= -1.f) return (1.f - z) * (1.f - z);
            return -4.f * z;
        }
        case L_SQUARED: { float d = p - y; return 0.5f * d * d; }
        case L_QUANTILE: {
            float e = y - p;
            return e > 0.f ? P.quantile_tau * e : (P.quantile_tau - 1.f) * e;
        }
        case L_EPS_INSENSITIVE: { float z = fabsf(y - p) - P.epsilon; return z > 0.f ? z : 0.f; }
        case L_SQ_EPS_INSENSITIVE: { float z = fabsf(y - p) - P.epsilon; return z > 0.f ? z * z : 0.f; }
        case L_HUBER: {
            float r = fabsf(p - y);
            return r <= P.huber_c ? 0.5f * r * r : P.huber_c * (r - 0.5f * P.huber_c);
        }
    }
    return 0.f;
}

HM_HD float loss_dloss(int l, float p, float y, const Params& P) {
    switch (l) {
        case L_HINGE: return y * p < 1.f ? -y : 0.f;
        case L_LOG: {
            float z = y * p;
            if (z > 18.f) return -y * expf(-z);
            if (z < -18.f) return -y;
            return -y / (1.f + expf(z));
        }
        case L_SQUARED_HINGE: { float z = 1.f - y * p; return z > 0.f ? -2.f * y * z : 0.f; }
        case L_MODIFIED_HUBER: {
            float z = y * p;
            if (z >= 1.f) return 0.f;
            if (z >= -1.f) return -2.f * y * (1.f - z);
            return -4.f * y;
        }
        case L_SQUARED: return p - y;
        case L_QUANTILE: return y > p ? -P.quantile_tau : (1.f - P.quantile_tau);
        case L_EPS_INSENSITIVE: {
            float e = y - p;
            return fabsf(e) > P.epsilon ? -sgnf(e) : 0.f;
        }
        case L_SQ_EPS_INSENSITIVE: {
            float e = y - p, z = fabsf(e) - P.epsilon;
            return z > 0.f ? -2.f * sgnf(e) * z : 0.f;
        }
        case L_HUBER: {
            float r = p - y;
            return fabsf(r) <= P.huber_c ? r : P.huber_c * sgnf(r);
        }
    }
    return 0.f;
}

// ---------------------------------------------------------------- eta schedules
HM_HD float eta_at(const Params& P, float t) {
    switch (P.eta) {
        case E_FIXED: return P.eta0;
        case E_SIMPLE: return P.total_steps > 0.f ? P.eta0 / (1.f + t / P.total_steps) : P.eta0;
        default: return P.eta0 / powf(t > 1.f ? t : 1.f, P.power_t);
    }
}

// Row-invariant step constants: the eta schedule and Adam-family bias corrections depend only on
// the step t, so each row computes them once (powf per feature update dominated the CPU engine:
// a9a AdaGrad 0.92 -> see docs/perf_notes.md) instead of once per feature.
struct StepK {
    float t, eta;
    float c1, c2, c1n, cp1, cp2;   // 1 - beta^t, 1 - beta2^t, 1 - beta1^(t+1), 1 - beta^(t-1) (Adam family)
};
HM_HD StepK step_consts(const Params& P, float t) {
    StepK k;
    k.t = t;
    k.eta = eta_at(P, t);
    const bool adam = P.opt == O_ADAM || P.opt == O_EVE || P.opt == O_ADAM_HD || P.opt == O_NADAM;
    k.c1 = adam ? 1.f - powf(P.beta1, t) : 0.f;
    k.c2 = adam ? 1.f - powf(P.beta2, t) : 0.f;
    k.c1n = P.opt == O_NADAM ? 1.f - powf(P.beta1, t + 1.f) : 0.f;
    k.cp1 = P.opt == O_ADAM_HD ? 1.f - powf(P.beta1, t - 1.f) : 0.f;
    k.cp2 = P.opt == O_ADAM_HD ? 1.f - powf(P.beta2, t - 1.f) : 0.f;
    return k;
}

// ---------------------------------------------------------------- regularisers
HM_HD float regularize(const Params& P, float w, float g) {
    switch (P.reg) {
        case R_L1: return g + P.lambda * sgnf(w);
        case R_L2: return g + P.lambda * w;
        case R_ELASTIC: return g + P.lambda * (P.l1_ratio * sgnf(w) + (1.f - P.l1_ratio) * w);
        default: return g;
    }
}

// ---------------------------------------------------------------- optimizers
// g is dloss * x_i (before regularisation); t >= 1 is the replica step counter.
HM_HD void optimizer_update(const Params& P, F4& s, float g, const StepK& k, float eve_d) {
    const int o = (P.reg == R_RDA && P.opt == O_ADAGRAD) ? O_ADAGRAD_RDA : P.opt;
    if (o != O_ADAGRAD_RDA) g = regularize(P, s.w, g);
    const float eta = k.eta;
    const float t = k.t;
    switch (o) {
        case O_SGD: s.w -= eta * g; break;
        case O_MOMENTUM: {
            s.s1 = P.beta1 * s.s1 + eta * g;   // beta1 doubles as the momentum (-momentum)
            s.w -= s.s1;
            break;
        }
        case O_NESTEROV: {
            const float prev = s.s1;
            s.s1 = P.beta1 * s.s1 - eta * g;
            s.w += -P.beta1 * prev + (1.f + P.beta1) * s.s1;
            break;
        }
        case O_ADAGRAD: {
            s.s1 += g * g;
            s.w -= eta * g / (sqrtf(s.s1) + P.eps);
            break;
        }
        case O_RMSPROP: {
            s.s1 = P.decay * s.s1 + (1.f - P.decay) * g * g;
            s.w -= eta * g / (sqrtf(s.s1) + P.eps);
            break;
        }
        case O_RMSPROP_GRAVES: {
            s.s1 = P.decay * s.s1 + (1.f - P.decay) * g * g;   // n
            s.s2 = P.decay * s.s2 + (1.f - P.decay) * g;       // g-bar
            const float den = s.s1 - s.s2 * s.s2 + P.eps;
            s.s3 = P.beta1 * s.s3 - eta * P.alpha * g / sqrtf(den > 0.f ? den : P.eps);  // delta
            s.w += s.s3;
            break;
        }
        case O_ADADELTA: {
            s.s1 = P.rho * s.s1 + (1.f - P.rho) * g * g;
            const float dx = sqrtf(s.s2 + P.eps) / sqrtf(s.s1 + P.eps) * g;
            s.s2 = P.rho * s.s2 + (1.f - P.rho) * dx * dx;
            s.w -= dx;
            break;
        }
        case O_ADAM:
        case O_EVE:
        case O_ADAM_HD: {
            const float m_prev = s.s1, v_prev = s.s2;
            s.s1 = P.beta1 * s.s1 + (1.f - P.beta1) * g;
            s.s2 = P.beta2 * s.s2 + (1.f - P.beta2) * g * g;
            const float c1 = k.c1, c2 = k.c2;
            float vhat = s.s2;
            if (o == O_ADAM && P.amsgrad) { s.s3 = fmaxf(s.s3, s.s2); vhat = s.s3; }
            float lr = eta * P.alpha * sqrtf(c2) / c1;
            if (o == O_EVE) lr /= (eve_d > 0.f ? eve_d : 1.f);
            if (o == O_ADAM_HD) {
                // per-coordinate hypergradient descent on the step size (s3 = alpha_i)
                if (s.s3 == 0.f) s.s3 = P.alpha;
                const float cp1 = k.cp1, cp2 = k.cp2;
                const float u_prev = (t > 1.f && cp1 > 0.f)
                                         ? (m_prev / cp1) / (sqrtf(v_prev / (cp2 > 0.f ? cp2 : 1.f)) + P.eps)
                                         : 0.f;
                s.s3 += P.beta_hd * g * u_prev;
                lr = eta * s.s3 * sqrtf(c2) / c1;
            }
            s.w -= lr * s.s1 / (sqrtf(vhat) + P.eps);
            break;
        }
        case O_NADAM: {
            s.s1 = P.beta1 * s.s1 + (1.f - P.beta1) * g;
            s.s2 = P.beta2 * s.s2 + (1.f - P.beta2) * g * g;
            const float c1 = k.c1, c1n = k.c1n;
            const float c2 = k.c2;
            const float mhat = P.beta1 * s.s1 / c1n + (1.f - P.beta1) * g / c1;
            const float vhat = s.s2 / c2;
            s.w -= eta * P.alpha * mhat / (sqrtf(vhat) + P.eps);
            break;
        }
        case O_ADAGRAD_RDA: {
            // AdaGrad + RDA (Duchi et al. 2011): s1 = sum of gradients u, s2 = sum of squares G
            s.s1 += g;
            s.s2 += g * g;
            const float sign = s.s1 > 0.f ? 1.f : -1.f;
            const float mean = sign * s.s1 / t - P.lambda;
            s.w = mean < 0.f ? 0.f : -sign * eta * t * mean / sqrtf(s.s2);
            break;
        }
    }
}

// ---------------------------------------------------------------- row-level coefficients
// What the per-row pass needs to gather: score p (always), xᵀΣx (covariance algorithms),
// ‖x‖² (PA family).
HM_HD bool needs_var(int algo) {
    return algo == A_CW || algo == A_AROW || algo == A_AROWH || algo == A_SCW1 || algo == A_SCW2 ||
           algo == A_AROW_REGR || algo == A_AROWE_REGR || algo == A_AROWE2_REGR;
}
HM_HD bool has_covar(int algo) { return needs_var(algo); }

struct RowCoef {
    int update;     // 0: skip the feature pass
    float a;        // w += a * (covar-weighted) x  (binary/regression rules)
    float b;        // covariance step (AROW/SCW beta, CW gamma*phi)
    float dloss;    // general learners: dloss(p, y)
    float loss;     // per-row loss for the convergence check
};

HM_HD float cw_gamma(float margin, float var, float phi) {
    const float b = 1.f + 2.f * phi * margin;
    const float den = 4.f * phi * var;
    if (den == 0.f) return 0.f;
    const float disc = b * b - 8.f * phi * (margin - phi * var);
    const float num = -b + sqrtf(disc > 0.f ? disc : 0.f);
    return num / den;
}

HM_HD void scw_alpha_beta(int algo, float m, float v, float phi, float C, float* alpha, float* beta) {
    const float phi2 = phi * phi;
    float a;
    if (algo == A_SCW1) {
        const float psi = 1.f + phi2 * 0.5f, zeta = 1.f + phi2;
        const float disc = m * m * phi2 * phi2 * 0.25f + v * phi2 * zeta;
        a = (-m * psi + sqrtf(disc > 0.f ? disc : 0.f)) / (v * zeta);
        a = a > 0.f ? a : 0.f;
        a = a < C ? a : C;
    } else {
        const float n = v + 0.5f / C;
        const float gamma = phi * sqrtf(phi2 * m * m * v * v + 4.f * n * v * (n + v * phi2));
        a = (-(2.f * m * n + phi2 * m * v) + gamma) / (2.f * (n * n + n * v * phi2));
        a = a > 0.f ? a : 0.f;
    }
    const float q = -a * v * phi + sqrtf(a * a * v * v * phi2 + 4.f * v);
    const float u = 0.25f * q * q;
    *alpha = a;
    *beta = a * phi / (sqrtf(u) + v * a * phi);
}

// Binary / regression row rule.  p: score, y: label (+-1) or target, var: xᵀΣx, sq: ‖x‖².
// rs: the replica scalars (already advanced: rs[RS_T] is this row's step).
HM_HD RowCoef row_rule(const Params& P, float p, float y, float var, float sq, float* rs) {
    RowCoef c = {0, 0.f, 0.f, 0.f, 0.f};
    const float m = y * p;
    switch (P.algo) {
        case A_PERCEPTRON:
            c.loss = m <= 0.f ? 1.f : 0.f;
            if (m <= 0.f) { c.update = 1; c.a = y; }
            break;
        case A_PA: case A_PA1: case A_PA2: {
            const float l = 1.f - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f && sq > 0.f) {
                float eta = l / sq;
                if (P.algo == A_PA1) eta = eta < P.c ? eta : P.c;
                if (P.algo == A_PA2) eta = l / (sq + 0.5f / P.c);
                c.update = 1; c.a = eta * y;
            }
            break;
        }
        case A_CW: {
            const float g = cw_gamma(m, var, P.phi);
            c.loss = m < 0.f ? 1.f : 0.f;
            if (g > 0.f) { c.update = 1; c.a = g * y; c.b = 2.f * g * P.phi; }
            break;
        }
        case A_AROW: case A_AROWH: {
            const float th = P.algo == A_AROWH ? P.c : 1.f;
            const float l = th - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f) {
                const float beta = 1.f / (var + P.r);
                c.update = 1; c.a = l * beta * y; c.b = beta;
            }
            break;
        }
        case A_SCW1: case A_SCW2: {
            const float l = P.phi * sqrtf(var) - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f && var > 0.f) {
                float alpha, beta;
                scw_alpha_beta(P.algo, m, var, P.phi, P.c, &alpha, &beta);
                if (alpha > 0.f) { c.update = 1; c.a = alpha * y; c.b = beta; }
            }
            break;
        }
        case A_ADAGRAD_RDA: {
            const float l = 1.f - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f) { c.update = 1; c.dloss = -y; }
            break;
        }
        case A_LOGRESS: case A_ADAGRAD_REGR: case A_ADADELTA_REGR: {
            // logistic regression on a [0,1] target: gradient = target - sigmoid(p)
            const float s = sigmoidf(p);
            const float g = y - s;
            c.loss = -(y * logf(fmaxf(s, 1e-7f)) + (1.f - y) * logf(fmaxf(1.f - s, 1e-7f)));
            c.update = g != 0.f;
            c.dloss = -g;
            break;
        }
        case A_PA1_REGR: case A_PA2_REGR: case A_PA1A_REGR: case A_PA2A_REGR: {
            float eps = P.epsilon;
            if (P.algo == A_PA1A_REGR || P.algo == A_PA2A_REGR) {
                // adaptive epsilon: epsilon x stddev of the targets seen so far
                const float n = rs[RS_N] + 1.f;
                const float d = y - rs[RS_MEAN];
                rs[RS_MEAN] += d / n;
                rs[RS_M2] += d * (y - rs[RS_MEAN]);
                rs[RS_N] = n;
                const float sd = n > 1.f ? sqrtf(rs[RS_M2] / (n - 1.f)) : 0.f;
                eps = P.epsilon * sd;
            }
            const float e = y - p;
            const float l = fabsf(e) - eps;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f && sq > 0.f) {
                float eta;
                if (P.algo == A_PA1_REGR || P.algo == A_PA1A_REGR) { eta = l / sq; eta = eta < P.c ? eta : P.c; }
                else eta = l / (sq + 0.5f / P.c);
                c.update = 1; c.a = eta * sgnf(e);
            }
            break;
        }
        case A_AROW_REGR: case A_AROWE_REGR: case A_AROWE2_REGR: {
            const float e = y - p;
            float l = e;
            if (P.algo != A_AROW_REGR) {
                float eps = P.epsilon;
                if (P.algo == A_AROWE2_REGR) {
                    const float n = rs[RS_N] + 1.f;
                    const float d = y - rs[RS_MEAN];
                    rs[RS_MEAN] += d / n;
                    rs[RS_M2] += d * (y - rs[RS_MEAN]);
                    rs[RS_N] = n;
                    eps = P.epsilon * (n > 1.f ? sqrtf(rs[RS_M2] / (n - 1.f)) : 0.f);
                }
                const float z = fabsf(e) - eps;
                l = z > 0.f ? sgnf(e) * z : 0.f;
            }
            c.loss = fabsf(l);
            if (l != 0.f) {
                const float beta = 1.f / (var + P.r);
                c.update = 1; c.a = l * beta; c.b = beta;
            }
            break;
        }
        case A_GENERAL: {
            c.loss = loss_value(P.loss, p, y, P);
            c.dloss = loss_dloss(P.loss, p, y, P);
            c.update = c.dloss != 0.f;
            if (P.opt == O_EVE) {
                // Eve feedback (Koushik & Hayashi 2016), tracked on the per-row loss
                const float f = c.loss + 1e-8f;
                const float fp = rs[RS_EVE_F];
                if (fp > 0.f) {
                    float r = fabsf(f - fp) / fminf(f, fp);
                    r = fminf(fmaxf(r, 0.1f), 10.f);
                    rs[RS_EVE_D] = 0.999f * rs[RS_EVE_D] + 0.001f * r;
                } else {
                    rs[RS_EVE_D] = 1.f;
                }
                rs[RS_EVE_F] = f;
            }
            break;
        }
    }
    return c;
}

// Per-feature update of a binary/regression rule.  x: feature value, t: step.
HM_HD void feature_update(const Params& P, const RowCoef& c, F4& s, float x, const StepK& k, float eve_d) {
    const float t = k.t;
    switch (P.algo) {
        case A_PERCEPTRON: case A_PA: case A_PA1: case A_PA2:
        case A_PA1_REGR: case A_PA2_REGR: case A_PA1A_REGR: case A_PA2A_REGR:
            s.w += c.a * x;
            break;
        case A_CW: {
            s.w += c.a * s.s1 * x;
            s.s1 = 1.f / (1.f / s.s1 + c.b * x * x);
            break;
        }
        case A_AROW: case A_AROWH: case A_SCW1: case A_SCW2:
        case A_AROW_REGR: case A_AROWE_REGR: case A_AROWE2_REGR: {
            const float sx = s.s1 * x;
            s.w += c.a * sx;
            s.s1 -= c.b * sx * sx;
            break;
        }
        case A_ADAGRAD_RDA: {
            const float g = c.dloss * x;
            s.s1 += g;
            s.s2 += g * g;
            const float sign = s.s1 > 0.f ? 1.f : -1.f;
            const float mean = sign * s.s1 / t - P.lambda;
            s.w = mean < 0.f ? 0.f : -sign * P.eta0 * t * mean / sqrtf(s.s2);
            break;
        }
        case A_LOGRESS: {
            s.w -= k.eta * c.dloss * x;
            break;
        }
        case A_ADAGRAD_REGR: {
            const float g = -c.dloss * x;  // ascent direction (target - sigmoid)
            s.s1 += g * g;
            s.w += P.eta0 * g / sqrtf(P.eps + s.s1);
            break;
        }
        case A_ADADELTA_REGR: {
            const float g = -c.dloss * x;
            s.s1 = P.rho * s.s1 + (1.f - P.rho) * g * g;
            const float dx = sqrtf(s.s2 + P.eps) / sqrtf(s.s1 + P.eps) * g;
            s.s2 = P.rho * s.s2 + (1.f - P.rho) * dx * dx;
            s.w += dx;
            break;
        }
        case A_GENERAL:
            optimizer_update(P, s, c.dloss * x, k, eve_d);
            break;
    }
}

// ---------------------------------------------------------------- multiclass
// Row rule on (actual label score sa, best wrong label score sm, variances va, vm).
struct MCCoef {
    int update;
    float a_act, a_miss;   // w_actual += a_act * (Σ)x ; w_missed += a_miss * (Σ)x
    float b;               // covariance step
    float loss;
};

HM_HD MCCoef mc_rule(const Params& P, float sa, float sm, float va, float vm, float sq) {
    MCCoef c = {0, 0.f, 0.f, 0.f, 0.f};
    const float m = sa - sm;
    switch (P.algo) {
        case A_PERCEPTRON:
            c.loss = m <= 0.f ? 1.f : 0.f;
            if (m <= 0.f) { c.update = 1; c.a_act = 1.f; c.a_miss = -1.f; }
            break;
        case A_PA: case A_PA1: case A_PA2: {
            const float l = 1.f - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f && sq > 0.f) {
                float eta = l / (2.f * sq);
                if (P.algo == A_PA1) eta = eta < P.c ? eta : P.c;
                if (P.algo == A_PA2) eta = l / (2.f * sq + 0.5f / P.c);
                c.update = 1; c.a_act = eta; c.a_miss = -eta;
            }
            break;
        }
        case A_CW: {
            const float var = va + vm;
            const float g = cw_gamma(m, var, P.phi);
            c.loss = m < 0.f ? 1.f : 0.f;
            if (g > 0.f) { c.update = 1; c.a_act = g; c.a_miss = -g; c.b = 2.f * g * P.phi; }
            break;
        }
        case A_AROW: case A_AROWH: {
            const float th = P.algo == A_AROWH ? P.c : 1.f;
            const float l = th - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f) {
                const float beta = 1.f / (va + vm + P.r);
                c.update = 1; c.a_act = l * beta; c.a_miss = -l * beta; c.b = beta;
            }
            break;
        }
        case A_SCW1: case A_SCW2: {
            const float var = va + vm;
            const float l = P.phi * sqrtf(var) - m;
            c.loss = l > 0.f ? l : 0.f;
            if (l > 0.f && var > 0.f) {
                float alpha, beta;
                scw_alpha_beta(P.algo, m, var, P.phi, P.c, &alpha, &beta);
                if (alpha > 0.f) { c.update = 1; c.a_act = alpha; c.a_miss = -alpha; c.b = beta; }
            }
            break;
        }
    }
    return c;
}

HM_HD void mc_feature_update(const Params& P, float a, float b, F4& s, float x) {
    if (has_covar(P.algo)) {
        if (P.algo == A_CW) {
            s.w += a * s.s1 * x;
            s.s1 = 1.f / (1.f / s.s1 + b * x * x);
        } else {
            const float sx = s.s1 * x;
            s.w += a * sx;
            s.s1 -= b * sx * sx;
        }
    } else {
        s.w += a * x;
    }
}

}  // namespace hm_lin
