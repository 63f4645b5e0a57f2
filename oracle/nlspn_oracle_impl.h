/*
 * ORACLE BODY — test infrastructure only; never linked into the product path.
 *
 * Precision-generic body of the CPU restatement of NLSPN's propagation section.
 * Included twice by nlspn_oracle.c, once with REAL=float (suffix _f32) and once
 * with REAL=double (suffix _f64).  Every function cites the reference lines it
 * restates (paths relative to the reference repo root).
 *
 * Arithmetic is written in the reference's own operation order so that, built
 * with -ffp-contract=off, the float instance is the exact IEEE sequence the
 * reference issues (modulo the order ATen/BLAS picks for its sums, which the
 * reference does not pin; sums here run over the tap/channel index in order).
 */

/* nlspnmodel.py:179-201 (_affinity_normalization) + :261-269 (_aff_insert).
 * aff_raw: B x K planes of HW, batch stride aff_bstride (elements).
 * aff_out: B x (K+1) planes of HW, contiguous; reference tap at K/2. */
void FN(orc_aff_norm)(const REAL *aff_raw, long long aff_bstride, int B, int K,
                      long long HW, int kind, REAL gamma, REAL *aff_out)
{
    const int ref = K / 2;                        /* nlspnmodel.py:91 idx_ref */
    const long long ob = (long long)(K + 1) * HW;
#pragma omp parallel for num_threads(orc_threads) schedule(static)
    for (long long bp = 0; bp < (long long)B * HW; ++bp) {
        const long long b = bp / HW, p = bp % HW;
        REAL t[64];
        REAL s = 0;
        for (int k = 0; k < K; ++k) {
            REAL a = aff_raw[b * aff_bstride + k * HW + p];
            if (kind == ORC_TC)                   /* :182-183 tanh(aff)/gamma */
                a = TANH(a) / gamma;
            else if (kind == ORC_TGASS)           /* :184-185 tanh(aff)/(gamma+1e-8) */
                a = TANH(a) / (gamma + (REAL)1e-8);
            t[k] = a;
        }
        for (int k = 0; k < K; ++k)               /* :190-191 sum |aff| (+1e-4 below) */
            s += FABS(t[k]);
        s = s + (REAL)1e-4;
        if (kind == ORC_ASS || kind == ORC_TGASS) /* :193-194 clamp sum to >= 1 */
            if (s < (REAL)1.0) s = (REAL)1.0;
        if (kind != ORC_TC)                       /* :196-197 divide (AS/ASS/TGASS) */
            for (int k = 0; k < K; ++k) t[k] = t[k] / s;
        REAL sum = 0;                             /* :262-263 aff_ref = 1 - sum(aff) */
        for (int k = 0; k < K; ++k) sum += t[k];
        REAL aref = (REAL)1.0 - sum;
        REAL *o = aff_out + b * ob + p;
        for (int k = 0, c = 0; c < K + 1; ++c) {  /* :265-267 insert at idx_ref */
            if (c == ref) o[c * HW] = aref;
            else o[c * HW] = t[k++];
        }
    }
}

/* nlspnmodel.py:252-259 (_off_insert): view (B,K,2,H,W), insert a zero (dh,dw)
 * pair at tap idx_ref -> (B, 2(K+1), H, W). */
void FN(orc_off_insert)(const REAL *off_raw, long long off_bstride, int B, int K,
                        long long HW, REAL *off_out)
{
    const int ref = K / 2;
    for (int b = 0; b < B; ++b)
        for (int c = 0, k = 0; c < K + 1; ++c) {
            REAL *o = off_out + ((long long)b * 2 * (K + 1) + 2 * c) * HW;
            if (c == ref) {
                for (long long p = 0; p < 2 * HW; ++p) o[p] = 0;
            } else {
                const REAL *s = off_raw + b * off_bstride + 2LL * k * HW;
                for (long long p = 0; p < 2 * HW; ++p) o[p] = s[p];
                ++k;
            }
        }
}

/* modulated_deform_im2col_cuda.cuh:24-54 (mdmcn_im2col_bilinear), zero
 * contribution from out-of-image corners. */
static REAL FN(orc_bilinear)(const REAL *im, int H, int W, REAL h, REAL w)
{
    int h_low = (int)FLOOR(h);
    int w_low = (int)FLOOR(w);
    int h_high = h_low + 1;
    int w_high = w_low + 1;
    REAL lh = h - h_low;
    REAL lw = w - w_low;
    REAL hh = 1 - lh, hw = 1 - lw;
    REAL v1 = 0, v2 = 0, v3 = 0, v4 = 0;
    if (h_low >= 0 && w_low >= 0) v1 = im[(long long)h_low * W + w_low];
    if (h_low >= 0 && w_high <= W - 1) v2 = im[(long long)h_low * W + w_high];
    if (h_high <= H - 1 && w_low >= 0) v3 = im[(long long)h_high * W + w_low];
    if (h_high <= H - 1 && w_high <= W - 1) v4 = im[(long long)h_high * W + w_high];
    REAL w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
    return (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
}

/* Modulated DCNv2 forward specialised to NLSPN's use: channels = out channels = 1,
 * stride 1, dilation 1, deformable_group 1, weight all ones, bias zero
 * (nlspnmodel.py:107-121, :205-207).
 *   modulated_deform_im2col_cuda.cuh:127-194: per tap (i,j) in row-major order,
 *     h_im = (y - pad_h + i) + dh, w_im = (x - pad_w + j) + dw, sampled only if
 *     h_im > -1 && w_im > -1 && h_im < H && w_im < W, col = val * mask;
 *   modulated_deform_conv_cuda.cu:108-114: out = bias + sum_t col_t * weight_t.
 * off: B x 2*kh*kw planes (dh plane 2t, dw plane 2t+1); mask: B x kh*kw planes. */
void FN(orc_mdcn_c1)(const REAL *im, const REAL *off, const REAL *mask,
                     int B, int H, int W, int kh, int kw, int ph, int pw, REAL *out)
{
    const long long HW = (long long)H * W;
    const int KK = kh * kw;
#pragma omp parallel for collapse(2) num_threads(orc_threads) schedule(static)
    for (int b = 0; b < B; ++b)
        for (int y = 0; y < H; ++y) {
            const REAL *imb = im + b * HW;
            const REAL *offb = off + (long long)b * 2 * KK * HW;
            const REAL *mb = mask + (long long)b * KK * HW;
            for (int x = 0; x < W; ++x) {
                const long long p = (long long)y * W + x;
                REAL acc = 0;
                for (int i = 0; i < kh; ++i)
                    for (int j = 0; j < kw; ++j) {
                        const int t = i * kw + j;
                        const REAL dh = offb[(2LL * t) * HW + p];
                        const REAL dw = offb[(2LL * t + 1) * HW + p];
                        const REAL m = mb[(long long)t * HW + p];
                        REAL val = 0;
                        const REAL h_im = (y - ph + i) + dh;
                        const REAL w_im = (x - pw + j) + dw;
                        if (h_im > -1 && w_im > -1 && h_im < H && w_im < W)
                            val = FN(orc_bilinear)(imb, H, W, h_im, w_im);
                        acc += val * m;
                    }
                out[b * HW + p] = acc;
            }
        }
}

/* nlspnmodel.py:209-224: no-offset branch. Replicate pad by 1, the 9 shifted
 * slices in row-major (dy,dx) order, times aff (B,9,H,W), summed over taps.
 * The reference hard-codes 3x3 here regardless of prop_kernel. */
void FN(orc_prop_noffset)(const REAL *feat, const REAL *aff, int B, int H, int W, REAL *out)
{
    const long long HW = (long long)H * W;
#pragma omp parallel for collapse(2) num_threads(orc_threads) schedule(static)
    for (int b = 0; b < B; ++b)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const REAL *fb = feat + b * HW;
                const REAL *ab = aff + (long long)b * 9 * HW;
                REAL acc = 0;
                for (int t = 0; t < 9; ++t) {
                    int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
                    yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
                    xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
                    acc += fb[(long long)yy * W + xx] * ab[(long long)t * HW + (long long)y * W + x];
                }
                out[b * HW + (long long)y * W + x] = acc;
            }
}

static REAL FN(orc_clamp0)(REAL v) { return v < 0 ? (REAL)0 : v; }  /* torch.clamp(min=0) */

/* The whole propagation section, nlspnmodel.py:323-381:
 *   :323-325 off = _off_insert(off); aff = _affinity_normalization(aff)
 *   :328-334 mask_fix = (dep > 0); conf = (1-m)*conf + m
 *   :340-363 T iterations of  p = propagate_once(p*conf, off, aff);
 *            p = (1-m)*p + m*dep;  clamp if always_clip;  list_pred.append(p)
 *            (k == 1 first applies the blend/clamp to pred_init, :341-348)
 *   :375-377 pred = clamp(p, 0) unless always_clip.
 * off_raw == NULL selects the no-offset branch (3x3 replicate, K must be 8).
 * Returns 0 on success, nonzero on invalid arguments. */
int FN(orc_propagate)(const REAL *pred_init, const REAL *dep, const REAL *conf,
                      const REAL *aff_raw, long long aff_bstride,
                      const REAL *off_raw, long long off_bstride,
                      REAL gamma, int kind, int kh, int kw, int T, unsigned flags,
                      int B, int H, int W,
                      REAL *pred_inter, REAL *pred, REAL *aff_out, REAL *off_out, REAL *conf_out)
{
    const long long HW = (long long)H * W, N = (long long)B * HW;
    const int K = kh * kw - 1;
    const int preserve = (flags & ORC_PRESERVE) != 0;
    const int clip = (flags & ORC_ALWAYS_CLIP) != 0;
    if (K < 1 || K > 63 || (kh % 2) == 0 || (kw % 2) == 0 || T < 1) return 1;
    if (off_raw == NULL && K != 8) return 2;
    if (preserve && dep == NULL) return 3;

    REAL *off_ins = NULL;
    if (off_raw) {
        off_ins = off_out ? off_out : (REAL *)malloc(sizeof(REAL) * 2 * (K + 1) * N);
        FN(orc_off_insert)(off_raw, off_bstride, B, K, HW, off_ins);
    }
    FN(orc_aff_norm)(aff_raw, aff_bstride, B, K, HW, kind, gamma, aff_out);

    REAL *cf = NULL;
    if (conf) {
        cf = conf_out ? conf_out : (REAL *)malloc(sizeof(REAL) * N);
        for (long long i = 0; i < N; ++i) {
            REAL c = conf[i];
            if (preserve) {
                REAL m = dep[i] > 0 ? (REAL)1 : (REAL)0;
                c = ((REAL)1.0 - m) * c + m;
            }
            cf[i] = c;
        }
    }

    REAL *p = (REAL *)malloc(sizeof(REAL) * N);
    REAL *f = (REAL *)malloc(sizeof(REAL) * N);
    for (long long i = 0; i < N; ++i) {
        REAL v = pred_init[i];
        if (preserve) {
            REAL m = dep[i] > 0 ? (REAL)1 : (REAL)0;
            v = ((REAL)1.0 - m) * v + m * dep[i];
        }
        if (clip) v = FN(orc_clamp0)(v);
        p[i] = v;
    }
    for (int k = 0; k < T; ++k) {
        for (long long i = 0; i < N; ++i) f[i] = cf ? p[i] * cf[i] : p[i];
        if (off_ins)
            FN(orc_mdcn_c1)(f, off_ins, aff_out, B, H, W, kh, kw, (kh - 1) / 2, (kw - 1) / 2, p);
        else
            FN(orc_prop_noffset)(f, aff_out, B, H, W, p);
        REAL *o = pred_inter + (long long)k * N;
        for (long long i = 0; i < N; ++i) {
            REAL v = p[i];
            if (preserve) {
                REAL m = dep[i] > 0 ? (REAL)1 : (REAL)0;
                v = ((REAL)1.0 - m) * v + m * dep[i];
            }
            if (clip) v = FN(orc_clamp0)(v);
            p[i] = v;
            o[i] = v;
        }
    }
    for (long long i = 0; i < N; ++i) pred[i] = clip ? p[i] : FN(orc_clamp0)(p[i]);

    free(p);
    free(f);
    if (off_ins && off_ins != off_out) free(off_ins);
    if (cf && cf != conf_out) free(cf);
    return 0;
}

/* ------------------------------------------------------------------ backward
 * Gradient of the propagation section (autograd of nlspnmodel.py:323-381 with the
 * DCN backward of modulated_deform_conv_cuda.cu:124-280):
 *   grad_mask  (col2im_coord mval, .cuh:304-307): sum col * bilinear(im, h, w)
 *   grad_offset(col2im_coord val,  .cuh:309-312): sum coordinate_weight * col * mask,
 *              coordinate weight mdmcn_get_coordinate_weight (.cuh:84-125)
 *   grad_input (col2im, .cuh:196-254): bilinear weight (mdmcn_get_gradient_weight,
 *              .cuh:57-81) * col * mask scattered to the 4 corners
 * with col = grad_output (NLSPN weight = 1).  The elementwise parts follow torch's
 * autograd: clamp(min=0) passes grad where x >= 0; abs -> sign; masked s[s<1]=1
 * blocks the gradient; tanh -> 1 - y^2.  Gradients of dep are not produced.
 * grad_inter (T x N) may be NULL; grad_off_raw/grad_conf/grad_gamma may be NULL. */
static REAL FN(orc_coord_weight)(REAL h, REAL w, int H, int W, const REAL *im, int dir)
{
    if (h <= -1 || h >= H || w <= -1 || w >= W) return 0;  /* .cuh:88-92 */
    int h_low = (int)FLOOR(h), w_low = (int)FLOOR(w);
    int h_high = h_low + 1, w_high = w_low + 1;
    REAL weight = 0;
    if (dir == 0) {
        if (h_low >= 0 && w_low >= 0) weight += -1 * (w_low + 1 - w) * im[(long long)h_low * W + w_low];
        if (h_low >= 0 && w_high <= W - 1) weight += -1 * (w - w_low) * im[(long long)h_low * W + w_high];
        if (h_high <= H - 1 && w_low >= 0) weight += (w_low + 1 - w) * im[(long long)h_high * W + w_low];
        if (h_high <= H - 1 && w_high <= W - 1) weight += (w - w_low) * im[(long long)h_high * W + w_high];
    } else {
        if (h_low >= 0 && w_low >= 0) weight += -1 * (h_low + 1 - h) * im[(long long)h_low * W + w_low];
        if (h_low >= 0 && w_high <= W - 1) weight += (h_low + 1 - h) * im[(long long)h_low * W + w_high];
        if (h_high <= H - 1 && w_low >= 0) weight += -1 * (h - h_low) * im[(long long)h_high * W + w_low];
        if (h_high <= H - 1 && w_high <= W - 1) weight += (h - h_low) * im[(long long)h_high * W + w_high];
    }
    return weight;
}

int FN(orc_propagate_backward)(const REAL *pred_init, const REAL *dep, const REAL *conf,
                               const REAL *aff_raw, long long aff_bstride,
                               const REAL *off_raw, long long off_bstride,
                               REAL gamma, int kind, int kh, int kw, int T, unsigned flags,
                               int B, int H, int W,
                               const REAL *grad_pred, const REAL *grad_inter,
                               REAL *grad_pred_init, REAL *grad_conf, REAL *grad_aff_raw,
                               REAL *grad_off_raw, REAL *grad_gamma)
{
    const long long HW = (long long)H * W, N = (long long)B * HW;
    const int K = kh * kw - 1, KK = K + 1, REF = K / 2;
    const int ph = (kh - 1) / 2, pw = (kw - 1) / 2;
    const int preserve = (flags & ORC_PRESERVE) != 0;
    const int clip = (flags & ORC_ALWAYS_CLIP) != 0;
    if (K < 1 || K > 63 || (kh % 2) == 0 || (kw % 2) == 0 || T < 1) return 1;
    if (off_raw == NULL && K != 8) return 2;

    /* forward recompute, keeping p_0..p_T and the pre-clamp values */
    REAL *aff = (REAL *)malloc(sizeof(REAL) * KK * N);
    REAL *offi = off_raw ? (REAL *)malloc(sizeof(REAL) * 2 * KK * N) : NULL;
    REAL *cf = (REAL *)malloc(sizeof(REAL) * N);
    REAL *m = (REAL *)malloc(sizeof(REAL) * N);
    REAL *p = (REAL *)malloc(sizeof(REAL) * (T + 1) * N);
    REAL *pre = (REAL *)malloc(sizeof(REAL) * (T + 1) * N);
    REAL *f = (REAL *)malloc(sizeof(REAL) * N);
    FN(orc_aff_norm)(aff_raw, aff_bstride, B, K, HW, kind, gamma, aff);
    if (offi) FN(orc_off_insert)(off_raw, off_bstride, B, K, HW, offi);
    for (long long i = 0; i < N; ++i) {
        m[i] = preserve ? (dep[i] > 0 ? (REAL)1 : (REAL)0) : (REAL)0;
        REAL c = conf ? conf[i] : (REAL)1;
        if (conf && preserve) c = ((REAL)1.0 - m[i]) * c + m[i];
        cf[i] = c;
        REAL v = pred_init[i];
        if (preserve) v = ((REAL)1.0 - m[i]) * v + m[i] * dep[i];
        pre[i] = v;
        p[i] = clip ? FN(orc_clamp0)(v) : v;
    }
    for (int t = 1; t <= T; ++t) {
        const REAL *pp = p + (long long)(t - 1) * N;
        for (long long i = 0; i < N; ++i) f[i] = conf ? pp[i] * cf[i] : pp[i];
        REAL *o = p + (long long)t * N, *pr = pre + (long long)t * N;
        if (offi) FN(orc_mdcn_c1)(f, offi, aff, B, H, W, kh, kw, ph, pw, o);
        else FN(orc_prop_noffset)(f, aff, B, H, W, o);
        for (long long i = 0; i < N; ++i) {
            REAL v = o[i];
            if (preserve) v = ((REAL)1.0 - m[i]) * v + m[i] * dep[i];
            pr[i] = v;
            o[i] = clip ? FN(orc_clamp0)(v) : v;
        }
    }

    /* reverse sweep */
    REAL *gaff = (REAL *)calloc((size_t)KK * N, sizeof(REAL));
    REAL *goff = (REAL *)calloc((size_t)2 * KK * N, sizeof(REAL));
    REAL *gcf = (REAL *)calloc((size_t)N, sizeof(REAL));
    REAL *gp = (REAL *)calloc((size_t)N, sizeof(REAL)); /* dL/dp_t */
    REAL *gf = (REAL *)calloc((size_t)N, sizeof(REAL)); /* dL/df_{t-1} */
    for (long long i = 0; i < N; ++i) {
        REAL g = grad_inter ? grad_inter[(long long)(T - 1) * N + i] : 0;
        if (grad_pred) g += clip ? grad_pred[i] : (p[(long long)T * N + i] >= 0 ? grad_pred[i] : 0);
        gp[i] = g;
    }
    for (int t = T; t >= 1; --t) {
        const REAL *pp = p + (long long)(t - 1) * N, *pr = pre + (long long)t * N;
        for (long long i = 0; i < N; ++i) f[i] = conf ? pp[i] * cf[i] : pp[i];
        for (long long i = 0; i < N; ++i) gf[i] = 0;
        for (int b = 0; b < B; ++b)
            for (int y = 0; y < H; ++y)
                for (int x = 0; x < W; ++x) {
                    const long long q = (long long)y * W + x, i = b * HW + q;
                    REAL g = gp[i];
                    if (clip && !(pr[i] >= 0)) g = 0;
                    const REAL go = preserve ? ((REAL)1.0 - m[i]) * g : g;
                    const REAL *fb = f + b * HW;
                    REAL *gfb = gf + b * HW;
                    for (int tap = 0; tap < KK; ++tap) {
                        const int ii = tap / kw, jj = tap % kw;
                        const REAL a = aff[((long long)b * KK + tap) * HW + q];
                        REAL hs, ws;
                        if (offi) {
                            hs = (y - ph + ii) + offi[((long long)b * 2 * KK + 2 * tap) * HW + q];
                            ws = (x - pw + jj) + offi[((long long)b * 2 * KK + 2 * tap + 1) * HW + q];
                        } else { /* replicate padding: clamp the integer sample point */
                            int yy = y + ii - 1, xx = x + jj - 1;
                            yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
                            xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
                            hs = yy; ws = xx;
                        }
                        if (!(hs > -1 && ws > -1 && hs < H && ws < W)) continue;
                        const REAL val = FN(orc_bilinear)(fb, H, W, hs, ws);
                        gaff[((long long)b * KK + tap) * HW + q] += go * val;           /* mval */
                        if (offi) {
                            goff[((long long)b * 2 * KK + 2 * tap) * HW + q] +=
                                FN(orc_coord_weight)(hs, ws, H, W, fb, 0) * go * a;     /* .cuh:309 */
                            goff[((long long)b * 2 * KK + 2 * tap + 1) * HW + q] +=
                                FN(orc_coord_weight)(hs, ws, H, W, fb, 1) * go * a;
                        }
                        const REAL top = go * a;                                          /* .cuh:236 */
                        const int hl = (int)FLOOR(hs), wl = (int)FLOOR(ws);
                        const REAL lh = hs - hl, lw = ws - wl, hh = 1 - lh, hw = 1 - lw;
                        if (hl >= 0 && wl >= 0) gfb[(long long)hl * W + wl] += hh * hw * top;
                        if (hl >= 0 && wl + 1 <= W - 1) gfb[(long long)hl * W + wl + 1] += hh * lw * top;
                        if (hl + 1 <= H - 1 && wl >= 0) gfb[(long long)(hl + 1) * W + wl] += lh * hw * top;
                        if (hl + 1 <= H - 1 && wl + 1 <= W - 1) gfb[(long long)(hl + 1) * W + wl + 1] += lh * lw * top;
                    }
                }
        /* f_{t-1} = p_{t-1} * conf' ; p_{t-1} = clamp(blend(...)) */
        for (long long i = 0; i < N; ++i) {
            if (conf) gcf[i] += gf[i] * pp[i];
            REAL g = conf ? gf[i] * cf[i] : gf[i];
            if (t - 1 >= 1 && grad_inter) g += grad_inter[(long long)(t - 2) * N + i];
            gp[i] = g;
        }
    }
    /* p_0 = clamp(blend(pred_init)) */
    for (long long i = 0; i < N; ++i) {
        REAL g = gp[i];
        if (clip && !(pre[i] >= 0)) g = 0;
        grad_pred_init[i] = preserve ? ((REAL)1.0 - m[i]) * g : g;
        if (grad_conf) grad_conf[i] = conf ? (preserve ? ((REAL)1.0 - m[i]) * gcf[i] : gcf[i]) : 0;
    }
    /* _off_insert backward: drop the reference pair */
    if (grad_off_raw && offi)
        for (int b = 0; b < B; ++b)
            for (int k = 0; k < K; ++k) {
                const int tap = k < REF ? k : k + 1;
                for (long long q = 0; q < 2 * HW; ++q)
                    grad_off_raw[((long long)b * 2 * K + 2 * k) * HW + q] = goff[((long long)b * 2 * KK + 2 * tap) * HW + q];
            }
    /* _aff_insert + _affinity_normalization backward */
    REAL gg = 0;
    for (int b = 0; b < B; ++b)
        for (long long q = 0; q < HW; ++q) {
            REAL u[64], G[64], th[64];
            const REAL gref = gaff[((long long)b * KK + REF) * HW + q];
            REAL s = 0;
            for (int k = 0; k < K; ++k) {
                const int tap = k < REF ? k : k + 1;
                G[k] = gaff[((long long)b * KK + tap) * HW + q] - gref;          /* aff_ref = 1 - sum */
                const REAL a = aff_raw[b * aff_bstride + k * HW + q];
                th[k] = TANH(a);
                u[k] = kind == ORC_TC ? th[k] / gamma : (kind == ORC_TGASS ? th[k] / (gamma + (REAL)1e-8) : a);
                s += FABS(u[k]);
            }
            s = s + (REAL)1e-4;
            const int clamped = (kind == ORC_ASS || kind == ORC_TGASS) && s < (REAL)1.0;
            const REAL se = clamped ? (REAL)1.0 : s;
            REAL dot = 0;
            for (int k = 0; k < K; ++k) dot += G[k] * u[k];
            for (int k = 0; k < K; ++k) {
                REAL gu;
                if (kind == ORC_TC) gu = G[k];
                else {
                    gu = G[k] / se;
                    if (!clamped) {
                        const REAL sg = u[k] > 0 ? (REAL)1 : (u[k] < 0 ? (REAL)-1 : (REAL)0);
                        gu += -dot / (se * se) * sg;
                    }
                }
                REAL ga = gu;
                if (kind == ORC_TC) ga = gu * (1 - th[k] * th[k]) / gamma;
                else if (kind == ORC_TGASS) {
                    const REAL d = gamma + (REAL)1e-8;
                    ga = gu * (1 - th[k] * th[k]) / d;
                    gg += -gu * th[k] / (d * d);
                }
                grad_aff_raw[((long long)b * K + k) * HW + q] = ga;
            }
        }
    if (grad_gamma) *grad_gamma = kind == ORC_TGASS ? gg : 0;

    free(aff); free(offi); free(cf); free(m); free(p); free(pre); free(f);
    free(gaff); free(goff); free(gcf); free(gp); free(gf);
    return 0;
}

/* ---------------------------------------------------------------------------
 * Generic modulated DCNv2 (seam 2 of the drop-in: the `DCN` module,
 * src/model/deformconv/src/vision.cpp:9-10).  Any channels / groups /
 * deformable groups / stride / padding / dilation.  Layouts as the reference:
 *   input (B,C,H,W), weight (Cout, C/group, kh, kw), bias (Cout) or NULL,
 *   offset (B, dg*2*kh*kw, Ho, Wo) [tap t: planes 2t (dh), 2t+1 (dw) of its group],
 *   mask (B, dg*kh*kw, Ho, Wo), output (B, Cout, Ho, Wo).
 * The sums the reference hands to BLAS (addmm / mm / addmv) are restated as plain
 * sums in index order (BLAS order is unspecified; compared within tolerance).
 * ------------------------------------------------------------------------- */

/* im2col value (.cuh:127-194): val(b, c, t, ho, wo) * mask, with h_in/w_in from
 * the given pads. */
static REAL FN(orc_im2col_val)(const REAL *in, const REAL *off, const REAL *mask, int b, int c, int t,
                               int ho, int wo, int C, int H, int W, int Ho, int Wo, int kw, int KK,
                               int sh, int sw, int ph, int pw, int dh, int dw, int dg, int cpdg,
                               REAL *inv_h_out, REAL *inv_w_out, REAL *m_out)
{
    const long long P = (long long)Ho * Wo, p = (long long)ho * Wo + wo;
    const int dgi = c / cpdg, i = t / kw, j = t % kw;
    const REAL oh = off[((long long)(b * dg + dgi) * 2 * KK + 2 * t) * P + p];
    const REAL ow = off[((long long)(b * dg + dgi) * 2 * KK + 2 * t + 1) * P + p];
    const REAL m = mask[((long long)(b * dg + dgi) * KK + t) * P + p];
    const REAL h_im = (ho * sh - ph + i * dh) + oh;  /* int + int, then + offset (.cuh:178-179) */
    const REAL w_im = (wo * sw - pw + j * dw) + ow;
    REAL val = 0;
    if (h_im > -1 && w_im > -1 && h_im < H && w_im < W)
        val = FN(orc_bilinear)(in + ((long long)b * C + c) * H * W, H, W, h_im, w_im);
    if (inv_h_out) *inv_h_out = h_im;
    if (inv_w_out) *inv_w_out = w_im;
    if (m_out) *m_out = m;
    return val * m;
}

/* forward: im2col + per-group addmm(bias, columns^T, weight^T) (.cu:90-116) */
void FN(orc_mdcn_fwd)(const REAL *in, const REAL *wt, const REAL *bias, const REAL *off, const REAL *mask,
                      int B, int C, int H, int W, int Cout, int kh, int kw, int sh, int sw, int ph, int pw,
                      int dh, int dw, int group, int dg, REAL *out)
{
    const int Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1, Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
    const int KK = kh * kw, cpg = C / group, opg = Cout / group, cpdg = C / dg;
    const long long P = (long long)Ho * Wo;
#pragma omp parallel for collapse(2) num_threads(orc_threads) schedule(static)
    for (int b = 0; b < B; ++b)
        for (int co = 0; co < Cout; ++co) {
            const int g = co / opg;
            for (long long p = 0; p < P; ++p) {
                const int ho = (int)(p / Wo), wo = (int)(p % Wo);
                REAL acc = 0;
                for (int cl = 0; cl < cpg; ++cl)
                    for (int t = 0; t < KK; ++t) {
                        const REAL col = FN(orc_im2col_val)(in, off, mask, b, g * cpg + cl, t, ho, wo, C, H, W, Ho, Wo,
                                                            kw, KK, sh, sw, ph, pw, dh, dw, dg, cpdg, 0, 0, 0);
                        acc += col * wt[((long long)co * cpg + cl) * KK + t];
                    }
                out[((long long)b * Cout + co) * P + p] = bias ? acc + bias[co] : acc;
            }
        }
}

/* mdmcn_get_gradient_weight (.cuh:57-81) */
static REAL FN(orc_grad_weight)(REAL ah, REAL aw, int h, int w, int H, int W)
{
    if (ah <= -1 || ah >= H || aw <= -1 || aw >= W) return 0;
    const int hl = (int)FLOOR(ah), wl = (int)FLOOR(aw), hh = hl + 1, wh = wl + 1;
    REAL weight = 0;
    if (h == hl && w == wl) weight = (h + 1 - ah) * (w + 1 - aw);
    if (h == hl && w == wh) weight = (h + 1 - ah) * (aw + 1 - w);
    if (h == hh && w == wl) weight = (ah + 1 - h) * (w + 1 - aw);
    if (h == hh && w == wh) weight = (ah + 1 - h) * (aw + 1 - w);
    return weight;
}

/* backward (.cu:124-280): columns = weight_g^T . grad_output_g per group; then
 * col2im_coord (.cuh:256-328) -> grad_offset, grad_mask; col2im (.cuh:196-254) ->
 * grad_input, with the reference's pad_w := pad_h at its call site (.cuh:371);
 * im2col again -> grad_weight += grad_output_g . columns_g^T; grad_bias +=
 * grad_output_g . ones.  grad_bias may be NULL.  Returns 0, or -1 on allocation
 * failure. */
int FN(orc_mdcn_bwd)(const REAL *in, const REAL *wt, const REAL *off, const REAL *mask, const REAL *go,
                     int B, int C, int H, int W, int Cout, int kh, int kw, int sh, int sw, int ph, int pw,
                     int dh, int dw, int group, int dg, REAL *g_in, REAL *g_off, REAL *g_mask, REAL *g_wt,
                     REAL *g_bias)
{
    const int Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1, Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
    const int KK = kh * kw, cpg = C / group, opg = Cout / group, cpdg = C / dg;
    const long long P = (long long)Ho * Wo, BP = (long long)B * P, HW = (long long)H * W;
    REAL *col = (REAL *)malloc(sizeof(REAL) * (size_t)C * KK * (size_t)BP);
    if (!col) return -1;
    /* columns (.cu:213-220) */
    for (int c = 0; c < C; ++c) {
        const int g = c / cpg, cl = c % cpg;
        for (int t = 0; t < KK; ++t)
            for (int b = 0; b < B; ++b)
                for (long long p = 0; p < P; ++p) {
                    REAL s = 0;
                    for (int ol = 0; ol < opg; ++ol) {
                        const int co = g * opg + ol;
                        s += wt[((long long)co * cpg + cl) * KK + t] * go[((long long)b * Cout + co) * P + p];
                    }
                    col[((long long)c * KK + t) * BP + (long long)b * P + p] = s;
                }
    }
    /* col2im_coord (.cuh:256-328) */
    for (int b = 0; b < B; ++b)
        for (int dgi = 0; dgi < dg; ++dgi)
            for (int oc = 0; oc < 2 * KK; ++oc)
                for (long long p = 0; p < P; ++p) {
                    const int t = oc / 2, dir = oc % 2, ho = (int)(p / Wo), wo = (int)(p % Wo);
                    REAL val = 0, mval = 0;
                    for (int cnt = 0; cnt < cpdg; ++cnt) {
                        const int c = dgi * cpdg + cnt;
                        const REAL cv = col[((long long)c * KK + t) * BP + (long long)b * P + p];
                        REAL ih, iw, m;
                        FN(orc_im2col_val)(in, off, mask, b, c, t, ho, wo, C, H, W, Ho, Wo, kw, KK, sh, sw, ph, pw,
                                           dh, dw, dg, cpdg, &ih, &iw, &m);
                        const REAL *im = in + ((long long)b * C + c) * HW;
                        if (ih <= -1 || iw <= -1 || ih >= H || iw >= W) {
                            ih = iw = -2;
                        } else {
                            mval += cv * FN(orc_bilinear)(im, H, W, ih, iw);
                        }
                        const REAL weight = FN(orc_coord_weight)(ih, iw, H, W, im, dir);
                        val += weight * cv * m;
                    }
                    g_off[((long long)(b * dg + dgi) * 2 * KK + oc) * P + p] = val;
                    if (dir == 0) g_mask[((long long)(b * dg + dgi) * KK + t) * P + p] = mval;
                }
    /* col2im (.cuh:196-254), pad_w := pad_h as the reference's call passes it */
    memset(g_in, 0, sizeof(REAL) * (size_t)B * C * HW);
    for (int c = 0; c < C; ++c)
        for (int t = 0; t < KK; ++t)
            for (int b = 0; b < B; ++b)
                for (long long p = 0; p < P; ++p) {
                    const int ho = (int)(p / Wo), wo = (int)(p % Wo);
                    REAL ih, iw, m;
                    FN(orc_im2col_val)(in, off, mask, b, c, t, ho, wo, C, H, W, Ho, Wo, kw, KK, sh, sw, ph, ph, dh,
                                       dw, dg, cpdg, &ih, &iw, &m);
                    const REAL top = col[((long long)c * KK + t) * BP + (long long)b * P + p] * m;
                    const int ch = (int)ih, cw = (int)iw;
                    for (int dy = -2; dy <= 2; ++dy)
                        for (int dx = -2; dx <= 2; ++dx) {
                            const int y = ch + dy, x = cw + dx;
                            if (y >= 0 && y < H && x >= 0 && x < W && FABS(ih - y) < 1 && FABS(iw - x) < 1) {
                                const REAL weight = FN(orc_grad_weight)(ih, iw, y, x, H, W);
                                g_in[((long long)b * C + c) * HW + (long long)y * W + x] += weight * top;
                            }
                        }
                }
    /* grad_weight / grad_bias (.cu:262-273) */
    for (int co = 0; co < Cout; ++co) {
        const int g = co / opg;
        for (int cl = 0; cl < cpg; ++cl)
            for (int t = 0; t < KK; ++t) {
                REAL s = 0;
                for (int b = 0; b < B; ++b)
                    for (long long p = 0; p < P; ++p)
                        s += go[((long long)b * Cout + co) * P + p] *
                             FN(orc_im2col_val)(in, off, mask, b, g * cpg + cl, t, (int)(p / Wo), (int)(p % Wo), C, H,
                                                W, Ho, Wo, kw, KK, sh, sw, ph, pw, dh, dw, dg, cpdg, 0, 0, 0);
                g_wt[((long long)co * cpg + cl) * KK + t] = s;
            }
        if (g_bias) {
            REAL s = 0;
            for (int b = 0; b < B; ++b)
                for (long long p = 0; p < P; ++p) s += go[((long long)b * Cout + co) * P + p];
            g_bias[co] = s;
        }
    }
    free(col);
    return 0;
}
