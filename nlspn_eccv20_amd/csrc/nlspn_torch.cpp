// Torch operator layer of the drop-in (SURVEY §8b "Build's exported surface", layer 2):
// the propagation path registered as torch ops in the `nlspn` namespace, so
// torch.ops.nlspn.* run with the dispatcher's own argument marshalling (no ctypes on
// the hot path), and TorchScript / torch.compile see them (fake kernels for shape
// propagation are registered in nlspn_eccv20_amd/ops.py).
//
// The reference binds its CUDA extension through pybind
// (src/model/deformconv/src/vision.cpp:6-13: modulated_deform_conv_forward /
// _backward).  Here every op is a thin host shim over the C ABI of
// include/nlspn_prop.h (libnlspn_hip.so): shape and dtype checks with the
// reference's message classes (TORCH_CHECK -> c10::Error -> Python RuntimeError,
// as AT_ASSERTM in modulated_deform_conv_cuda.cu:39-73), outputs allocated from the
// caching allocator, work enqueued on the current stream of the input's device.
//
//   nlspn::affinity_normalization  nlspnmodel.py:179-201 + _aff_insert :261-269
//   nlspn::prop_step               one fused iteration, :350-361 around _propagate_once :203-226
//   nlspn::propagate               the propagation section :323-381 (inference; the autograd
//                                  form stays nlspn_eccv20_amd.propagate)
//   nlspn::modulated_deform_conv_forward / _backward   seam 2, vision.cpp:9-10
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <string>
#include <tuple>
#include <vector>

#include "../../include/nlspn_prop.h"

namespace {

using at::Tensor;
using c10::optional;

void check_rc(int rc, const char *what) { TORCH_CHECK(rc == NLSPN_OK, what, ": ", nlspn_last_error()); }

void *stream_of(const Tensor &t) {
    hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index());
    return reinterpret_cast<void *>(s);
}

int prop_dtype(const Tensor &t) {
    if (t.scalar_type() == at::kFloat) return NLSPN_DTYPE_F32;
    if (t.scalar_type() == at::kHalf) return NLSPN_DTYPE_F16;
    TORCH_CHECK(false, "NLSPN propagation supports float32 and float16 storage, got ", t.scalar_type());
}

void check_cuda(const char *name, const Tensor &t) { TORCH_CHECK(t.is_cuda(), name, " must be a CUDA tensor"); }
void check_cuda(const char *name, const optional<Tensor> &t) {
    if (t.has_value()) check_cuda(name, *t);
}
// An operand of an op whose kernels index every operand as `ref`'s element type on
// `ref`'s device (the reference's data<scalar_t>() raises on a mismatch).
void check_like(const char *name, const Tensor &t, const Tensor &ref) {
    check_cuda(name, t);
    TORCH_CHECK(t.device() == ref.device(), name, " is on ", t.device(), ", expected ", ref.device());
    TORCH_CHECK(t.scalar_type() == ref.scalar_type(), name, " has dtype ", t.scalar_type(), ", expected ",
                ref.scalar_type());
}
void check_like(const char *name, const optional<Tensor> &t, const Tensor &ref) {
    if (t.has_value()) check_like(name, *t, ref);
}
const void *ptr(const optional<Tensor> &t) { return t.has_value() ? t->data_ptr() : nullptr; }
void *mut_ptr(optional<Tensor> &t) { return t.has_value() ? t->data_ptr() : nullptr; }

// (B, C, H, W) with contiguous H*W planes, consecutive within a batch item; returns the
// batch stride in elements (a channel slice of a larger head output is accepted).
int64_t planes(const char *name, const Tensor &t, int64_t B, int64_t C, int64_t H, int64_t W) {
    TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(2) == H && t.size(3) == W && (C < 0 || t.size(1) == C),
                name, " has shape ", t.sizes(), ", expected (", B, ", ", C < 0 ? std::string("*") : std::to_string(C),
                ", ", H, ", ", W, ")");
    TORCH_CHECK(t.stride(3) == 1 && (H == 1 || t.stride(2) == W) && (t.size(1) == 1 || t.stride(1) == H * W), name,
                " tensor has to have contiguous H*W planes");
    return B > 1 ? t.stride(0) : t.size(1) * H * W;
}

int aff_kind(const std::string &k) {
    if (k == "AS") return NLSPN_AFF_AS;
    if (k == "ASS") return NLSPN_AFF_ASS;
    if (k == "TC") return NLSPN_AFF_TC;
    if (k == "TGASS") return NLSPN_AFF_TGASS;
    TORCH_CHECK_NOT_IMPLEMENTED(false, "affinity ", k);
}

Tensor gamma_f32(const Tensor &gamma) {
    check_cuda("gamma", gamma);
    return gamma.detach().reshape({-1}).slice(0, 0, 1).to(at::kFloat).contiguous();
}

Tensor affinity_normalization(const Tensor &aff, const Tensor &gamma, const std::string &kind) {
    check_cuda("aff", aff);
    TORCH_CHECK(aff.dim() == 4, "aff must be (B, K, H, W)");
    const int64_t B = aff.size(0), K = aff.size(1), H = aff.size(2), W = aff.size(3);
    const int64_t bs = planes("aff", aff, B, K, H, W);
    const Tensor g = gamma_f32(gamma);
    Tensor out = at::empty({B, K + 1, H, W}, aff.options());
    c10::DeviceGuard guard(aff.device());
    check_rc(nlspn_affinity_normalize(prop_dtype(aff), aff.data_ptr(), bs, g.data_ptr<float>(), out.data_ptr(),
                                      (int)B, (int)K, (int)H, (int)W, aff_kind(kind), stream_of(aff)),
             "nlspn::affinity_normalization");
    return out;
}

Tensor prop_step(const Tensor &feat, const optional<Tensor> &confidence, const optional<Tensor> &dep,
                 const Tensor &aff, const optional<Tensor> &offset, int64_t kh, int64_t kw, bool raw_offsets,
                 bool preserve_input, bool always_clip) {
    check_cuda("feat", feat);
    check_cuda("confidence", confidence);
    check_cuda("dep", dep);
    check_like("aff", aff, feat);
    check_like("offset", offset, feat);
    check_like("confidence", confidence, feat);
    check_like("dep", dep, feat);
    TORCH_CHECK(kh % 2 == 1 && kw % 2 == 1, "only odd kernel is supported but k_f = ", kh, "x", kw);
    const int64_t K = kh * kw - 1;
    TORCH_CHECK(feat.dim() == 4, "feat must be (B, 1, H, W)");
    const int64_t B = feat.size(0), H = feat.size(2), W = feat.size(3);
    planes("feat", feat, B, 1, H, W);
    TORCH_CHECK(feat.is_contiguous(), "input tensor has to be contiguous");
    for (const auto &nt : {std::make_pair("confidence", &confidence), std::make_pair("dep", &dep)}) {
        if (nt.second->has_value()) {
            planes(nt.first, **nt.second, B, 1, H, W);
            TORCH_CHECK((*nt.second)->scalar_type() == feat.scalar_type() && (*nt.second)->is_contiguous(), nt.first,
                        " must be contiguous with feat's dtype");
        }
    }
    TORCH_CHECK(!preserve_input || dep.has_value(), "preserve_input requires dep");
    const int64_t abs = planes("aff", aff, B, K + 1, H, W);
    int64_t obs = 0;
    if (offset.has_value()) obs = planes("offset", *offset, B, raw_offsets ? 2 * K : 2 * (K + 1), H, W);
    Tensor out = at::empty_like(feat);
    const unsigned flags = (preserve_input ? NLSPN_PRESERVE_INPUT : 0u) | (always_clip ? NLSPN_ALWAYS_CLIP : 0u);
    c10::DeviceGuard guard(feat.device());
    check_rc(nlspn_prop_step(prop_dtype(feat), feat.data_ptr(), ptr(confidence), ptr(dep), aff.data_ptr(), abs,
                             ptr(offset), obs, raw_offsets ? NLSPN_OFF_RAW : NLSPN_OFF_INSERTED, out.data_ptr(), nullptr,
                             (int)B, (int)H, (int)W, (int)kh, (int)kw, flags, stream_of(feat)),
             "nlspn::prop_step");
    return out;
}

std::tuple<Tensor, Tensor, Tensor, optional<Tensor>, optional<Tensor>> propagate(
    const Tensor &pred_init, const optional<Tensor> &dep, const optional<Tensor> &confidence, const Tensor &aff,
    const optional<Tensor> &offset, const Tensor &gamma, int64_t prop_time, int64_t kh, int64_t kw,
    const std::string &affinity, bool preserve_input, bool always_clip) {
    check_cuda("pred_init", pred_init);
    check_cuda("dep", dep);
    check_cuda("confidence", confidence);
    check_cuda("aff", aff);
    check_cuda("offset", offset);
    TORCH_CHECK(kh % 2 == 1 && kw % 2 == 1, "only odd kernel is supported but k_f = ", kh, "x", kw);
    TORCH_CHECK(prop_time >= 1, "prop_time must be >= 1, got ", prop_time);
    const int64_t K = kh * kw - 1;
    TORCH_CHECK(pred_init.dim() == 4 && pred_init.size(1) == 1, "ch_f must equal pred_init.shape[1] == 1");
    const int64_t B = pred_init.size(0), H = pred_init.size(2), W = pred_init.size(3);
    planes("pred_init", pred_init, B, 1, H, W);
    TORCH_CHECK(pred_init.is_contiguous(), "pred_init must be contiguous");
    for (const auto &nt : {std::make_pair("dep", &dep), std::make_pair("confidence", &confidence)}) {
        if (nt.second->has_value()) {
            planes(nt.first, **nt.second, B, 1, H, W);
            TORCH_CHECK((*nt.second)->scalar_type() == pred_init.scalar_type() && (*nt.second)->is_contiguous(),
                        nt.first, " must be contiguous with pred_init's dtype");
        }
    }
    TORCH_CHECK(!preserve_input || dep.has_value(), "preserve_input requires dep");
    const int64_t abs = planes("aff", aff, B, K, H, W);
    const int64_t obs = offset.has_value() ? planes("offset", *offset, B, 2 * K, H, W) : 0;
    check_like("aff", aff, pred_init);
    check_like("offset", offset, pred_init);
    check_like("dep", dep, pred_init);
    check_like("confidence", confidence, pred_init);
    TORCH_CHECK(gamma.device() == pred_init.device(), "gamma is on ", gamma.device(), ", expected ",
                pred_init.device());
    const int dt = prop_dtype(pred_init);
    const Tensor g = gamma_f32(gamma);
    const auto o = pred_init.options();
    Tensor pred_inter = at::empty({prop_time, B, 1, H, W}, o);
    Tensor pred = at::empty({B, 1, H, W}, o);
    Tensor aff_out = at::empty({B, K + 1, H, W}, o);
    optional<Tensor> off_out, conf_out;
    if (offset.has_value()) off_out = at::empty({B, 2 * (K + 1), H, W}, o);
    if (confidence.has_value()) conf_out = at::empty({B, 1, H, W}, o);
    const size_t wsb = nlspn_workspace_bytes(dt, (int)B, (int)H, (int)W);
    Tensor ws = at::empty({(int64_t)((wsb + 3) / 4)}, o.dtype(at::kInt));
    const unsigned flags = (preserve_input ? NLSPN_PRESERVE_INPUT : 0u) | (always_clip ? NLSPN_ALWAYS_CLIP : 0u);
    c10::DeviceGuard guard(pred_init.device());
    TORCH_CHECK(nlspn_resident_status(1) == 0, "nlspn::propagate: ", nlspn_last_error());
    check_rc(nlspn_propagate(dt, pred_init.data_ptr(), ptr(dep), ptr(confidence), aff.data_ptr(), abs, ptr(offset),
                             obs, g.data_ptr<float>(), pred_inter.data_ptr(), pred.data_ptr(), aff_out.data_ptr(),
                             mut_ptr(off_out), mut_ptr(conf_out), ws.data_ptr(), (int)B, (int)H, (int)W, (int)kh, (int)kw,
                             (int)prop_time, aff_kind(affinity), flags, stream_of(pred_init)),
             "nlspn::propagate");
    return {pred, pred_inter, aff_out, off_out, conf_out};
}

// The propagation loop from prologued inputs (nlspnmodel.py:340-381; nlspn_propagate_normalized):
// p0 = the blended [clamped] pred_init, the blended confidence, the normalised (K+1)-tap
// affinity and the inserted 2(K+1)-plane offsets — what the fused head epilogue writes
// (heads.head_epilogue_prologue).  Inference only.  -> (pred, pred_inter (T,B,1,H,W))
std::tuple<Tensor, Tensor> propagate_normalized(const Tensor &p0, const optional<Tensor> &dep,
                                                const optional<Tensor> &confidence, const Tensor &aff,
                                                const Tensor &offset, int64_t prop_time, int64_t kh, int64_t kw,
                                                bool preserve_input, bool always_clip) {
    check_cuda("p0", p0);
    check_cuda("aff", aff);
    check_cuda("offset", offset);
    TORCH_CHECK(kh % 2 == 1 && kw % 2 == 1, "only odd kernel is supported but k_f = ", kh, "x", kw);
    TORCH_CHECK(prop_time >= 1, "prop_time must be >= 1, got ", prop_time);
    const int64_t K = kh * kw - 1;
    TORCH_CHECK(p0.dim() == 4 && p0.size(1) == 1, "p0 must be (B, 1, H, W)");
    const int64_t B = p0.size(0), H = p0.size(2), W = p0.size(3);
    for (const auto &nt : {std::make_pair("dep", &dep), std::make_pair("confidence", &confidence)})
        if (nt.second->has_value()) check_like(nt.first, *nt.second, p0);
    check_like("aff", aff, p0);
    check_like("offset", offset, p0);
    const auto exact = [&](const char *n, const Tensor &t, int64_t C) {
        TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == C && t.size(2) == H && t.size(3) == W &&
                        t.is_contiguous(),
                    n, " must be a contiguous (", B, ", ", C, ", ", H, ", ", W, ") tensor, got ", t.sizes());
    };
    exact("p0", p0, 1);
    if (dep.has_value()) exact("dep", *dep, 1);
    if (confidence.has_value()) exact("confidence", *confidence, 1);
    exact("aff", aff, K + 1);
    exact("offset", offset, 2 * (K + 1));
    TORCH_CHECK(!preserve_input || dep.has_value(), "preserve_input requires dep");
    const int dt = prop_dtype(p0);
    const auto o = p0.options();
    Tensor pred_inter = at::empty({prop_time, B, 1, H, W}, o);
    Tensor pred = at::empty({B, 1, H, W}, o);
    const size_t wsb = nlspn_workspace_bytes(dt, (int)B, (int)H, (int)W);
    Tensor ws = at::empty({(int64_t)((wsb + 3) / 4)}, o.dtype(at::kInt));
    const unsigned flags = (preserve_input ? NLSPN_PRESERVE_INPUT : 0u) | (always_clip ? NLSPN_ALWAYS_CLIP : 0u);
    c10::DeviceGuard guard(p0.device());
    TORCH_CHECK(nlspn_resident_status(1) == 0, "nlspn::propagate_normalized: ", nlspn_last_error());
    check_rc(nlspn_propagate_normalized(dt, p0.data_ptr(), ptr(dep), ptr(confidence), aff.data_ptr(), offset.data_ptr(),
                                        pred_inter.data_ptr(), pred.data_ptr(), ws.data_ptr(), (int)B, (int)H, (int)W,
                                        (int)kh, (int)kw, (int)prop_time, flags, stream_of(p0)),
             "nlspn::propagate_normalized");
    return {pred, pred_inter};
}

int dcn_dtype(const Tensor &t, bool backward) {
    if (t.scalar_type() == at::kFloat) return NLSPN_DTYPE_F32;
    if (t.scalar_type() == at::kDouble) return NLSPN_DTYPE_F64;
    TORCH_CHECK_NOT_IMPLEMENTED(!backward && t.scalar_type() == at::kHalf, "modulated_deform_conv: dtype ",
                                t.scalar_type(), " is not supported");
    return NLSPN_DTYPE_F16;
}

// DCN.modulated_deform_conv_forward (vision.cpp:9; modulated_deform_conv_cuda.cu:19-121)
Tensor mdcn_forward(const Tensor &input, const Tensor &weight, const optional<Tensor> &bias, const Tensor &offset,
                    const Tensor &mask, int64_t kernel_h, int64_t kernel_w, int64_t stride_h, int64_t stride_w,
                    int64_t pad_h, int64_t pad_w, int64_t dilation_h, int64_t dilation_w, int64_t group,
                    int64_t deformable_group, int64_t im2col_step) {
    (void)im2col_step;  // no columns buffer to chunk
    TORCH_CHECK(input.is_contiguous(), "input tensor has to be contiguous");
    TORCH_CHECK(weight.is_contiguous(), "weight tensor has to be contiguous");
    check_cuda("input", input);
    check_like("weight", weight, input);
    check_like("bias", bias, input);
    check_like("offset", offset, input);
    check_like("mask", mask, input);
    TORCH_CHECK(input.dim() == 4 && weight.dim() == 4, "input and weight must be 4-D");
    const int64_t B = input.size(0), C = input.size(1), H = input.size(2), W = input.size(3);
    const int64_t Cout = weight.size(0);
    TORCH_CHECK(weight.size(2) == kernel_h && weight.size(3) == kernel_w, "Input shape and kernel shape wont match: (",
                kernel_h, " x ", kernel_w, " vs ", weight.size(2), " x ", weight.size(3), ").");
    TORCH_CHECK(C == weight.size(1) * group, "Input shape and kernel channels wont match: (", C, " vs ",
                weight.size(1) * group, ").");
    const int64_t Ho = (H + 2 * pad_h - (dilation_h * (kernel_h - 1) + 1)) / stride_h + 1;
    const int64_t Wo = (W + 2 * pad_w - (dilation_w * (kernel_w - 1) + 1)) / stride_w + 1;
    const int64_t KK = kernel_h * kernel_w;
    TORCH_CHECK(offset.sizes() == at::IntArrayRef({B, 2 * deformable_group * KK, Ho, Wo}), "offset has shape ",
                offset.sizes());
    TORCH_CHECK(mask.sizes() == at::IntArrayRef({B, deformable_group * KK, Ho, Wo}), "mask has shape ", mask.sizes());
    const Tensor off_c = offset.contiguous(), mask_c = mask.contiguous();
    optional<Tensor> bias_c;
    if (bias.has_value()) bias_c = bias->contiguous();
    Tensor out = at::empty({B, Cout, Ho, Wo}, input.options());
    c10::DeviceGuard guard(input.device());
    check_rc(nlspn_mdcn_forward(dcn_dtype(input, false), input.data_ptr(), weight.data_ptr(), ptr(bias_c),
                                off_c.data_ptr(), mask_c.data_ptr(), out.data_ptr(), (int)B, (int)C, (int)H, (int)W,
                                (int)Cout, (int)kernel_h, (int)kernel_w, (int)stride_h, (int)stride_w, (int)pad_h,
                                (int)pad_w, (int)dilation_h, (int)dilation_w, (int)group, (int)deformable_group,
                                stream_of(input)),
             "nlspn::modulated_deform_conv_forward");
    return out;
}

// DCN.modulated_deform_conv_backward (vision.cpp:10; .cu:124-280): [grad_input,
// grad_offset, grad_mask, grad_weight, grad_bias]
std::vector<Tensor> mdcn_backward(const Tensor &input, const Tensor &weight, const Tensor &bias,
                                  const Tensor &offset, const Tensor &mask, const Tensor &grad_output,
                                  int64_t kernel_h, int64_t kernel_w, int64_t stride_h, int64_t stride_w,
                                  int64_t pad_h, int64_t pad_w, int64_t dilation_h, int64_t dilation_w, int64_t group,
                                  int64_t deformable_group, int64_t im2col_step) {
    (void)im2col_step;
    TORCH_CHECK(input.is_contiguous(), "input tensor has to be contiguous");
    TORCH_CHECK(weight.is_contiguous(), "weight tensor has to be contiguous");
    check_cuda("input", input);
    check_like("weight", weight, input);
    check_like("bias", bias, input);
    check_like("offset", offset, input);
    check_like("mask", mask, input);
    check_like("grad_output", grad_output, input);
    TORCH_CHECK(input.dim() == 4 && weight.dim() == 4, "input and weight must be 4-D");
    const int64_t B = input.size(0), C = input.size(1), H = input.size(2), W = input.size(3);
    const int64_t Cout = weight.size(0);
    const int64_t KK = kernel_h * kernel_w;
    TORCH_CHECK(weight.size(2) == kernel_h && weight.size(3) == kernel_w && C == weight.size(1) * group,
                "weight has shape ", weight.sizes());
    TORCH_CHECK(bias.numel() == Cout, "bias has ", bias.numel(), " elements, expected ", Cout);
    TORCH_CHECK(C % group == 0 && Cout % group == 0, "channels(", C, ") and channels_out(", Cout,
                ") must divide group(", group, ")");
    const int64_t Ho = (H + 2 * pad_h - (dilation_h * (kernel_h - 1) + 1)) / stride_h + 1;
    const int64_t Wo = (W + 2 * pad_w - (dilation_w * (kernel_w - 1) + 1)) / stride_w + 1;
    TORCH_CHECK(grad_output.sizes() == at::IntArrayRef({B, Cout, Ho, Wo}), "grad_out has shape ",
                grad_output.sizes());
    TORCH_CHECK(offset.sizes() == at::IntArrayRef({B, 2 * deformable_group * KK, Ho, Wo}), "offset has shape ",
                offset.sizes());
    TORCH_CHECK(mask.sizes() == at::IntArrayRef({B, deformable_group * KK, Ho, Wo}), "mask has shape ", mask.sizes());
    const Tensor off_c = offset.contiguous(), mask_c = mask.contiguous(), go = grad_output.contiguous();
    Tensor gi = at::empty_like(input), goff = at::empty_like(off_c), gm = at::empty_like(mask_c),
           gw = at::empty_like(weight);
    Tensor gb = at::empty_like(bias);
    c10::DeviceGuard guard(input.device());
    check_rc(nlspn_mdcn_backward(dcn_dtype(input, true), input.data_ptr(), weight.data_ptr(), off_c.data_ptr(),
                                 mask_c.data_ptr(), go.data_ptr(), gi.data_ptr(), goff.data_ptr(), gm.data_ptr(),
                                 gw.data_ptr(), gb.data_ptr(), (int)B, (int)C, (int)H,
                                 (int)W, (int)Cout, (int)kernel_h, (int)kernel_w, (int)stride_h, (int)stride_w,
                                 (int)pad_h, (int)pad_w, (int)dilation_h, (int)dilation_w, (int)group,
                                 (int)deformable_group, stream_of(input)),
             "nlspn::modulated_deform_conv_backward");
    return {gi, goff, gm, gw, gb};
}

}  // namespace

TORCH_LIBRARY(nlspn, m) {
    m.def("affinity_normalization(Tensor aff, Tensor gamma, str kind=\"TGASS\") -> Tensor");
    m.def("prop_step(Tensor feat, Tensor? confidence, Tensor? dep, Tensor aff, Tensor? offset, int kh=3, int kw=3, "
          "bool raw_offsets=False, bool preserve_input=True, bool always_clip=False) -> Tensor");
    m.def("propagate(Tensor pred_init, Tensor? dep, Tensor? confidence, Tensor aff, Tensor? offset, Tensor gamma, "
          "int prop_time=18, int kh=3, int kw=3, str affinity=\"TGASS\", bool preserve_input=True, "
          "bool always_clip=False) -> (Tensor, Tensor, Tensor, Tensor?, Tensor?)");
    m.def("propagate_normalized(Tensor p0, Tensor? dep, Tensor? confidence, Tensor aff, Tensor offset, "
          "int prop_time=18, int kh=3, int kw=3, bool preserve_input=True, bool always_clip=False) -> (Tensor, Tensor)");
    m.def("modulated_deform_conv_forward(Tensor input, Tensor weight, Tensor? bias, Tensor offset, Tensor mask, "
          "int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h, int pad_w, int dilation_h, "
          "int dilation_w, int group, int deformable_group, int im2col_step) -> Tensor");
    m.def("modulated_deform_conv_backward(Tensor input, Tensor weight, Tensor bias, Tensor offset, Tensor mask, "
          "Tensor grad_output, int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h, int pad_w, "
          "int dilation_h, int dilation_w, int group, int deformable_group, int im2col_step) -> Tensor[]");
}

// CPU tensors: the reference's own answer (modulated_deform_conv.h:43, :85) — there is
// no CPU path (the CPU oracle under oracle/ is test infrastructure, never this).
namespace {
[[noreturn]] void no_cpu() { TORCH_CHECK(false, "Not implemented on the CPU"); }
Tensor affnorm_cpu(const Tensor &, const Tensor &, const std::string &) { no_cpu(); }
Tensor prop_step_cpu(const Tensor &, const optional<Tensor> &, const optional<Tensor> &, const Tensor &,
                     const optional<Tensor> &, int64_t, int64_t, bool, bool, bool) {
    no_cpu();
}
std::tuple<Tensor, Tensor, Tensor, optional<Tensor>, optional<Tensor>> propagate_cpu(
    const Tensor &, const optional<Tensor> &, const optional<Tensor> &, const Tensor &, const optional<Tensor> &,
    const Tensor &, int64_t, int64_t, int64_t, const std::string &, bool, bool) {
    no_cpu();
}
std::tuple<Tensor, Tensor> propagate_normalized_cpu(const Tensor &, const optional<Tensor> &, const optional<Tensor> &,
                                                    const Tensor &, const Tensor &, int64_t, int64_t, int64_t, bool,
                                                    bool) {
    no_cpu();
}
Tensor mdcn_forward_cpu(const Tensor &, const Tensor &, const optional<Tensor> &, const Tensor &, const Tensor &,
                        int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                        int64_t) {
    no_cpu();
}
std::vector<Tensor> mdcn_backward_cpu(const Tensor &, const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                                      const Tensor &, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                                      int64_t, int64_t, int64_t, int64_t) {
    no_cpu();
}
}  // namespace

TORCH_LIBRARY_IMPL(nlspn, CPU, m) {
    m.impl("affinity_normalization", &affnorm_cpu);
    m.impl("prop_step", &prop_step_cpu);
    m.impl("propagate", &propagate_cpu);
    m.impl("propagate_normalized", &propagate_normalized_cpu);
    m.impl("modulated_deform_conv_forward", &mdcn_forward_cpu);
    m.impl("modulated_deform_conv_backward", &mdcn_backward_cpu);
}

TORCH_LIBRARY_IMPL(nlspn, CUDA, m) {
    m.impl("affinity_normalization", &affinity_normalization);
    m.impl("prop_step", &prop_step);
    m.impl("propagate", &propagate);
    m.impl("propagate_normalized", &propagate_normalized);
    m.impl("modulated_deform_conv_forward", &mdcn_forward);
    m.impl("modulated_deform_conv_backward", &mdcn_backward);
}
