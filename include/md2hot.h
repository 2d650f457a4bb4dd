/*
 * md2hot.h — C ABI of the MI355X (gfx950) monodepth2 photometric hot path.
 *
 * One fused operator replaces the body of
 *   Trainer.generate_images_pred   /root/reference/trainer.py:341-391
 *   Trainer.compute_losses         /root/reference/trainer.py:407-496
 *   (+ compute_reprojection_loss   trainer.py:393-405, and the layers.py
 *    primitives they call: disp_to_depth 16-25, BackprojectDepth 139-168,
 *    Project3D 171-193, get_smooth_loss 202-215, SSIM 218-248)
 * and the autograd backward of all of it (dL/ddisp_s for every scale and
 * dL/dcam_T_cam for every source frame).
 *
 * The reference exposes no FFI: its boundary is the two Python methods above.
 * This header is what the Python host side (monodepth2_amd/_lib.py, ctypes)
 * binds; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every tensor is fp32 (disparities: fp32 or bf16, md2_desc.disp_dtype),
 *    contiguous NCHW, device memory owned by the caller
 *    (PyTorch's caching allocator).  The library never allocates outside
 *    md2_aug_plan_create: scratch lives in `workspace` (md2_workspace_bytes) and
 *    must be the SAME buffer for a forward and its backward (the forward leaves
 *    per-image statistics there).
 *  - Work is enqueued on `stream` (a hipStream_t); no host synchronisation, no
 *    device malloc, so every call except md2_aug_run (host-staged parameters) is
 *    hipGraph-capturable.
 *  - Return 0 on success, a negative code otherwise; md2_last_error() then
 *    describes the failure (thread-local).  Nothing in the library aborts.
 *  - Results are deterministic: every reduction is a fixed-order tree.
 */
#ifndef MD2HOT_H
#define MD2HOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MD2_ABI_VERSION 23
#define MD2_MAX_SCALES 4
#define MD2_MAX_SRC 3

#define MD2_OK 0
#define MD2_ERR_ARG (-1)
#define MD2_ERR_HIP (-2)

/* opt.* switches of the reference (options.py:104-118) */
#define MD2_NO_SSIM          (1u << 0) /* --no_ssim             trainer.py:399-403      */
#define MD2_AVG_REPROJECTION (1u << 1) /* --avg_reprojection    trainer.py:441-442,461  */
#define MD2_NO_AUTOMASK      (1u << 2) /* --disable_automasking trainer.py:432,466,480  */
#define MD2_V1_MULTISCALE    (1u << 3) /* --v1_multiscale       trainer.py:347-352,417  */
#define MD2_T_PER_SCALE      (1u << 4) /* a cam_T_cam per scale (posecnn, trainer.py:366-375) */
#define MD2_PREDICTIVE_MASK  (1u << 5) /* --predictive_mask     trainer.py:447-459 (needs NO_AUTOMASK) */

/* md2_desc.disp_dtype: the disparities (and the gradients written for them) as fp32,
 * or bf16 as the depth decoder emits them under bf16 autocast (config C5), read as is */
#define MD2_DTYPE_F32  0u
#define MD2_DTYPE_BF16 1u

typedef struct md2_desc {
    int32_t batch;               /* B: images per rank (opt.batch_size)                  */
    int32_t height, width;       /* opt.height / opt.width (full resolution)             */
    int32_t num_src;             /* S = len(frame_ids) - 1, 1..3                          */
    int32_t num_scales;          /* len(opt.scales) (scales are 0..num_scales-1), 1..4   */
    uint32_t flags;              /* MD2_* above                                          */
    float min_depth, max_depth;  /* opt.min_depth / opt.max_depth                        */
    float disparity_smoothness;  /* opt.disparity_smoothness                             */
    uint32_t disp_dtype;         /* MD2_DTYPE_*: element type of disp[] and grad_disp[]  */
    uint64_t seed;               /* tie-break noise seed when tensors.noise == NULL      */
} md2_desc;

/*
 * Operands.  "loss resolution" of scale s is (H, W) normally and
 * (H>>s, W>>s) with MD2_V1_MULTISCALE (trainer.py:347-352).
 */
typedef struct md2_tensors {
    /* outputs[("disp", s)]: (B,1,H>>s,W>>s) */
    const float* disp[MD2_MAX_SCALES];
    /* inputs[("color", frame, s)]: (B,3,H>>s,W>>s); frame 0 = target (frame_ids[0]),
     * frames 1..S = frame_ids[1:].  Targets are read at every scale (smoothness,
     * trainer.py:423,488); sources only at the loss resolution of each scale. */
    const float* color[MD2_MAX_SCALES][1 + MD2_MAX_SRC];
    /* inputs[("K", s)] / inputs[("inv_K", s)]: (B,4,4); only [0] unless V1_MULTISCALE */
    const float* K[MD2_MAX_SCALES];
    const float* inv_K[MD2_MAX_SCALES];
    /* cam_T_cam per source frame, stacked: (S,B,4,4); with MD2_T_PER_SCALE
     * (num_scales,S,B,4,4).  The stereo frame passes inputs["stereo_T"]. */
    const float* T;
    /* Optional unit-normal tie-break noise (trainer.py:468), per scale packed
     * back to back, scale s shaped (B, C, h_s, w_s) with C = S (or 1 with
     * AVG_REPROJECTION) at the loss resolution.  NULL: drawn in-kernel from seed. */
    const float* noise;
    /* Optional device-side uint64 mixed into desc.seed at run time, so a captured
     * hipGraph draws fresh noise on every replay (the caller increments it). */
    const uint64_t* seed_ptr;
    /* MD2_PREDICTIVE_MASK: outputs["predictive_mask"][("disp", s)] upsampled to the
     * loss resolution (trainer.py:449-453), per scale packed back to back, scale s
     * shaped (B, S, h_s, w_s).  Multiplies each frame's reprojection loss. */
    const float* mask;
    /* Optional (ABI 20): the source frames' scale-0 colours as 8-bit RGBx dwords,
     * (S, B, H, W) uint32, byte c of a pixel = k with color[0][1+f][b][c][y][x] == k/255
     * exactly — what the loader's to_tensor makes of 8-bit images (mono_dataset.py:
     * 199-200), e.g. written by md2_aug_run2 as it decodes them.  NULL: the forward
     * packs them from the fp32 planes itself and checks every colour (pack_src8).  The
     * forward and the backward must see the same value. */
    const uint32_t* src8;
} md2_tensors;

int md2_abi_version(void);
const char* md2_last_error(void);
/* Hash of the sources the library was built from (monodepth2_amd/build.py
 * source_hash(): every .hip source, the headers, the flags and the target), so the
 * Python binding can refuse a prebuilt library that is stale for the tree. */
const char* md2_build_id(void);

/* Scratch needed by one forward + backward pair (bytes, 256-B aligned). */
size_t md2_workspace_bytes(const md2_desc* desc);

/* Bytes of the per-pixel selection map the forward writes (one uint8 per
 * loss-resolution pixel per scale, scales packed back to back). */
size_t md2_select_bytes(const md2_desc* desc);

/*
 * Forward.  Writes loss_out[0..num_scales-1] = losses["loss/s"] and
 * loss_out[num_scales] = losses["loss"] (trainer.py:492-495), and select_out:
 * per pixel the argmin index into torch.cat((identity, reprojection), 1)
 * (trainer.py:471-478); identity_selection = select > (C-1) (trainer.py:481).
 */
int md2_photometric_fwd(const md2_desc* desc, const md2_tensors* t,
                        float* loss_out, uint8_t* select_out,
                        void* workspace, void* stream);

/*
 * Backward.  grad_loss: device (num_scales+1) upstream gradients of loss_out.
 * Writes (overwrites) grad_disp[s] shaped like disp[s], and grad_T shaped like
 * T, and with MD2_PREDICTIVE_MASK grad_mask shaped like tensors.mask (dL/dmask
 * through trainer.py:455; the BCE term of 457-459 is the caller's).  select and
 * workspace must come from the matching forward.
 */
int md2_photometric_bwd(const md2_desc* desc, const md2_tensors* t,
                        const float* grad_loss, const uint8_t* select,
                        float* const* grad_disp, float* grad_T, float* grad_mask,
                        void* workspace, void* stream);

/*
 * Materialise what generate_images_pred stores in `outputs` (trainer.py:356,
 * 382, 384-387) for logging / evaluation steps.  Any pointer may be NULL.
 *   depth_out[s]          (B,1,h_s,w_s)           outputs[("depth", 0, s)]
 *   sample_out[s*S + f]   (B,h_s,w_s,2)           outputs[("sample", frame, s)]
 *   color_out[s*S + f]    (B,3,h_s,w_s)           outputs[("color", frame, s)]
 */
int md2_generate_images(const md2_desc* desc, const md2_tensors* t,
                        float* const* depth_out, float* const* sample_out,
                        float* const* color_out, void* stream);

/*
 * The tie-break noise the forward draws in-kernel when tensors.noise is NULL
 * (trainer.py:468, unit normal before the 1e-5 scale), for scale s: writes
 * (B, C, h_s, w_s) with C = S (or 1 with AVG_REPROJECTION) at the loss resolution.
 * seed_ptr: the same optional device seed the forward takes.  Lets tests hand the exact draw of a
 * seeded forward to the CPU oracle.
 */
int md2_tiebreak_noise(const md2_desc* desc, const uint64_t* seed_ptr, int scale,
                       float* out, void* stream);

/*
 * Optional kernel timing for benchmarks: between md2_timing_begin and
 * md2_timing_end every launch of the photometric kernels (the forward's three
 * launches — identity, reprojection, combine — as one interval, and the backward
 * photo kernel; they dominate the hot path) is launched with hipExtLaunchKernelGGL,
 * which stamps a start/stop hipEvent pair on the kernel dispatches themselves (v1_multiscale's per-scale launches are not timed).
 * md2_timing_end waits
 * for the last event and returns the summed durations (ms) and launch counts.
 * Not for use under graph capture (events are recorded eagerly).
 */
int md2_timing_begin(int max_launches);
int md2_timing_end(double* fwd_ms, int* n_fwd, double* bwd_ms, int* n_bwd);
/* After md2_timing_end: the summed durations of whole md2_photometric_fwd calls (first
 * kernel's start to the finalize kernel's end) and md2_photometric_bwd calls (photo_bwd
 * start to grad_T end) in that window — every kernel of the hot path, for its roofline.
 * Each whole call takes a slot of max_launches besides its kernel slot. */
int md2_timing_calls(double* fwd_ms, int* n_fwd, double* bwd_ms, int* n_bwd);

/*
 * DepthDecoder block fusion: the input of every decoder
 * conv — ReflectionPad2d(1) (layers.py:127-135) of [ELU(previous conv output)
 * (layers.py:113-118), nearest x2 upsampled (layers.py:196-199), concatenated with
 * the encoder skip feature (networks/depth_decoder.py:55-58)] — in one pass, and its
 * adjoint in one pass.  x: (B,C,h,w); skip: (B,Cs,H,W) with (H,W) = (2h,2w) if
 * MD2_PAD_UPSAMPLE else (h,w); out: (B,C+Cs,H+2,W+2).  With MD2_PAD_ELU x is the
 * pre-activation and the backward needs it again.  Returns MD2_OK / MD2_ERR_*.
 */
#define MD2_PAD_ELU      (1u << 0)
#define MD2_PAD_UPSAMPLE (1u << 1)
#define MD2_PAD_NHWC     (1u << 2)   /* x, skip, out (and their grads) channels_last */
#define MD2_PAD_BF16     (1u << 3)   /* bf16 tensors (needs NHWC, channels multiples of 4) */

typedef struct md2_pad_desc {
    int32_t batch, channels, height, width; /* of x */
    int32_t skip_channels;                  /* 0: no skip tensor */
    uint32_t flags;                         /* MD2_PAD_* */
} md2_pad_desc;

/* bias (nullable, (C,) fp32): the bias of the conv that produced x, added here
 * before the ELU so the conv runs without one (no separate bias-add pass); the
 * backward then also returns grad_bias = the fixed-order sum of grad_x over
 * (B, h, w), with `workspace` of md2_decoder_pad_workspace_bytes.  NHWC with
 * channels a multiple of 4 dividing 1024 (every DepthDecoder width), else MD2_ERR_ARG. */
size_t md2_decoder_pad_workspace_bytes(const md2_pad_desc* desc);
int md2_decoder_pad_fwd(const md2_pad_desc* desc, const float* x, const float* skip, const float* bias,
                        float* out, void* stream);
int md2_decoder_pad_bwd(const md2_pad_desc* desc, const float* x, const float* bias, const float* grad_out,
                        float* grad_x, float* grad_skip, float* grad_bias, void* workspace, void* stream);
/* md2_decoder_pad_bwd of grad_out + grad_out2 (NULL = none; same shape and layout as
 * grad_out, MD2_PAD_NHWC with channel counts multiple of 4 only): the padded input of
 * upconv(i,1)'s output feeds both dispconv(i) and upconv(i-1,0) (depth_decoder.py:56-64),
 * so its two gradients are summed as they are read instead of by a separate add.
 * (ABI 19) */
int md2_decoder_pad_bwd2(const md2_pad_desc* desc, const float* x, const float* bias, const float* grad_out,
                         const float* grad_out2, float* grad_x, float* grad_skip, float* grad_bias, void* workspace,
                         void* stream);

/*
 * DepthDecoder disparity heads (networks/depth_decoder.py:63-64, layers.py:121-136):
 * disp = sigmoid(Conv2d(C, 1, 3)(padded) + bias) on the reflection-padded NHWC fp32
 * input that md2_decoder_pad_fwd builds, padded = (B, h+2, w+2, C); disp (B,1,h,w).
 * weight is the (1,C,3,3) parameter in its own memory format (MD2_HEAD_WEIGHT_CL:
 * channels_last, i.e. [ky][kx][c]; else [c][ky][kx]); grad_weight is written in the
 * same format.  The backward takes the forward's disp (sigmoid backward from its
 * output, as torch) and returns grad_padded (B,h+2,w+2,C) plus grad_weight /
 * grad_bias as fixed-order sums (deterministic), with `workspace` of
 * md2_disp_head_workspace_bytes.  C a multiple of 4 dividing 1024, C <= 256.
 * Replaces the dispconv Conv3x3 + nn.Sigmoid of the reference decoder.
 */
#define MD2_HEAD_WEIGHT_CL (1u << 0)
/* ABI 23: padded / grad_padded are bf16 (uint16 storage behind the float pointers; config
 * C5's bf16 decoder), widened exactly / rounded to nearest even; weight, bias, disp and
 * the gradients of the parameters stay fp32 */
#define MD2_HEAD_BF16 (1u << 1)

typedef struct md2_head_desc {
    int32_t batch, channels, height, width; /* of the unpadded output */
    uint32_t flags;                         /* MD2_HEAD_* */
} md2_head_desc;

size_t md2_disp_head_workspace_bytes(const md2_head_desc* desc);
int md2_disp_head_fwd(const md2_head_desc* desc, const float* padded, const float* weight, const float* bias,
                      float* disp, void* stream);
int md2_disp_head_bwd(const md2_head_desc* desc, const float* padded, const float* weight, const float* disp,
                      const float* grad_disp, float* grad_padded, float* grad_weight, float* grad_bias,
                      void* workspace, void* stream);

/*
 * Weight gradient of the ResNet stem convolution (conv1 of networks/resnet_encoder.py
 * via torchvision ResNet: Conv2d(C, 64, 7, stride 2, padding 3, bias=False)), whose
 * input is data (the normalised frames), so the input gradient is never needed.
 * x (batch, height, width, channels) NHWC fp32, channels 3 / 6 / 9 (one, two or three
 * frames); grad_y (batch, Ho, Wo, 64) NHWC with Ho = (height-1)/2+1, Wo likewise;
 * grad_weight (64, channels, 7, 7) written (not accumulated) in the weight's memory
 * format (MD2_STEM_WEIGHT_CL: channels_last [co][ky][kx][ci]; else [co][ci][ky][kx]).
 * Deterministic (fixed-order sums); workspace of md2_stem_wgrad_workspace_bytes.
 * Replaces MIOpen's backward-weights convolution for this layer.
 */
#define MD2_STEM_WEIGHT_CL (1u << 0)
/* ABI 23: bf16 operands (uint16 storage behind the float pointers; config C5's bf16
 * autocast stem), channels 3 / 6: md2_stem_wgrad's x and grad_y (grad_weight stays
 * fp32); md2_stem_fwd's x and y (the fp32 weight rounded to bf16, fp32 accumulation,
 * y rounded to nearest even) */
#define MD2_STEM_BF16 (1u << 1)

typedef struct md2_stem_desc {
    int32_t batch, channels, height, width; /* of the input */
    uint32_t flags;                         /* MD2_STEM_* */
} md2_stem_desc;

size_t md2_stem_wgrad_workspace_bytes(const md2_stem_desc* desc);
int md2_stem_wgrad(const md2_stem_desc* desc, const float* x, const float* grad_y, float* grad_weight,
                   void* workspace, void* stream);

/*
 * Forward of the same convolution: y (batch, Ho, Wo, 64) NHWC fp32 = conv(x, weight),
 * stride 2, padding 3, on split-bf16 MFMA (f32-class), channels 3 / 6.  weight
 * (64, channels, 7, 7) in the memory format MD2_STEM_WEIGHT_CL names.  No workspace.
 * Replaces MIOpen's forward convolution for this layer (torchvision conv1 forward,
 * networks/resnet_encoder.py:93).
 */
int md2_stem_fwd(const md2_stem_desc* desc, const float* x, const float* weight, float* y, void* stream);

/*
 * Conv bias (+ ReLU) epilogue on NHWC fp32 activations (networks/pose_decoder.py:43-54:
 * relu(conv(x) + b) and the last conv's bias), the convolution itself running
 * bias-free on MIOpen.  x / y / grad (pixels, channels) row-major = channels_last.
 * fwd: y = [relu](x + bias).
 * bwd: grad_x = grad_y · [y > 0] (MD2_BIAS_ACT_RELU only; without it grad_x is unused
 * and may be NULL) and grad_bias = Σ_pixels of that, in a fixed order, with `workspace`
 * of md2_bias_act_workspace_bytes.  channels a multiple of 4.
 */
#define MD2_BIAS_ACT_RELU (1u << 0)

typedef struct md2_bias_act_desc {
    int64_t pixels;
    int32_t channels;
    uint32_t flags; /* MD2_BIAS_ACT_* */
} md2_bias_act_desc;

int md2_bias_act_fwd(const md2_bias_act_desc* desc, const float* x, const float* bias, float* y, void* stream);
size_t md2_bias_act_workspace_bytes(const md2_bias_act_desc* desc);
int md2_bias_act_bwd(const md2_bias_act_desc* desc, const float* y, const float* grad_y, float* grad_x,
                     float* grad_bias, void* workspace, void* stream);

/*
 * The encoders' input (networks/resnet_encoder.py:93 normalisation, trainer.py:280-290
 * frame-pair concatenation) in one pass: src[g * slots + k] is a (batch,3,H,W) NCHW
 * fp32 frame tensor; out is (groups*batch, H, W, 3*slots) = a channels_last
 * (groups*batch, 3*slots, H, W) tensor with out = (src - mean) * (1.f / std) per channel
 * (torch's fp32 arithmetic for a division by a scalar).
 * groups * slots <= 8.  Returns MD2_OK / MD2_ERR_*.
 */
int md2_encoder_input(int groups, int batch, int slots, int height, int width, const float* const* src, float mean,
                      float std_, float* out, void* stream);

/*
 * The optimizer step (torch.optim.Adam as the reference's trainer.py:102-104, 209;
 * no weight decay / amsgrad) in one launch per 256 parameters over a device table of
 * chunks.  Every chunk is a contiguous run of n fp32 elements of one parameter with
 * its gradient and its two moment buffers in the same layout; `step` is the 1-based
 * step count the bias corrections use.  Returns MD2_OK / MD2_ERR_*.
 */
typedef struct md2_adam_chunk {
    float* p;         /* parameter elements [off, off + n) */
    float* m;         /* exp_avg, same elements */
    float* v;         /* exp_avg_sq, same elements */
    int64_t off;      /* element offset into the parameter's gradient */
    int64_t n;
    int32_t param;    /* index into grads[] */
    int32_t reserved;
} md2_adam_chunk;

/* table: device array of chunks ordered by param; chunk_start (host, nparams + 1):
 * first chunk of each parameter; grads (host, nparams): this step's gradient base
 * pointers (same layout as their parameters). */
int md2_adam_step(const md2_adam_chunk* table, const int* chunk_start, int nparams, const float* const* grads,
                  double lr, double beta1, double beta2, double eps, int step, void* stream);
/* The same step with the step counter and lr on the device (hipGraph-capturable, the
 * `capturable=True` form of torch.optim.Adam): *step (fp32, the value torch keeps in
 * state["step"]) is incremented first, the bias corrections are formed in double from
 * it and *lr (fp64, the param group's lr tensor that StepLR fills); `hyper` is 2 fp32
 * of device scratch. */
int md2_adam_step_dev(const md2_adam_chunk* table, const int* chunk_start, int nparams, const float* const* grads,
                      const double* lr, double beta1, double beta2, double eps, float* step, float* hyper,
                      void* stream);
/* The capturable step in parts (ABI v21): md2_adam_hyper advances *step and writes the
 * two factors to `hyper` (md2_adam_step_dev's first launch); md2_adam_apply_dev updates
 * the parameters [k_begin, k_end) of the table with them.  Calls over disjoint ranges,
 * each on a stream ordered after md2_adam_hyper and after its parameters' gradients,
 * cover the step once (the trainer runs the pose network's parameters on the pose
 * stream as soon as its backward is done).  grads is indexed like chunk_start. */
int md2_adam_hyper(const double* lr, double beta1, double beta2, float* step, float* hyper, void* stream);
int md2_adam_apply_dev(const md2_adam_chunk* table, const int* chunk_start, int k_begin, int k_end,
                       const float* const* grads, double beta1, double beta2, double eps, const float* hyper,
                       void* stream);

/*
 * Fused pose producer: transformation_from_parameters
 * (layers.py:28-45, with rot_from_axisangle 64-103 and get_translation_matrix
 * 48-61) for every (frame, image) of a step in one launch, and its adjoint.
 * axisangle, translation: (frames, batch, 3); T / grad_T: (frames, batch, 4, 4);
 * bit f of invert_mask selects invert=True for frame f (trainer.py:294-295).
 */
int md2_pose_fwd(int32_t frames, int32_t batch, uint32_t invert_mask, const float* axisangle,
                 const float* translation, float* T, void* stream);
int md2_pose_bwd(int32_t frames, int32_t batch, uint32_t invert_mask, const float* axisangle,
                 const float* translation, const float* grad_T, float* grad_axisangle,
                 float* grad_translation, void* stream);

/*
 * GPU input pipeline: what MonoDataset.__getitem__ does to
 * the decoded frames of a batch (datasets/mono_dataset.py:136-200 with
 * kitti_dataset.py:58-63) — horizontal flip, the cascaded Resize(ANTIALIAS) pyramid
 * (mono_dataset.py:80-84, 96-101), ToTensor and the per-item ColorJitter
 * (mono_dataset.py:66-78, 175-181, 103-108) — bit-exact with the PIL arithmetic the
 * reference runs on the CPU workers.  The per-item random decisions are drawn by the
 * caller (same draws, same order as the reference) and passed in `items`.
 */
typedef struct md2_aug_desc {
    int32_t items;                 /* batch size B */
    int32_t frames;                /* frames per item F (frame_ids, incl. "s") */
    int32_t in_height, in_width;   /* decoded frame size (scale -1) */
    int32_t height, width;         /* scale-0 size; scale s is (height>>s, width>>s) */
    int32_t num_scales;            /* 1..4 */
    int32_t reserved;
} md2_aug_desc;

#define MD2_AUG_BRIGHTNESS 0
#define MD2_AUG_CONTRAST   1
#define MD2_AUG_SATURATION 2
#define MD2_AUG_HUE        3

typedef struct md2_aug_item {
    uint8_t flip;        /* do_flip (mono_dataset.py:137): frames flipped left-right */
    uint8_t color_aug;   /* do_color_aug (mono_dataset.py:136) */
    uint8_t hue_shift;   /* np.uint8(hue_factor * 255), wrapped as numpy 1.x does */
    uint8_t reserved;
    uint8_t order[4];    /* MD2_AUG_* in application order (ColorJitter's shuffle) */
    float brightness, contrast, saturation;   /* the get_params factors */
} md2_aug_item;

typedef struct md2_aug_plan md2_aug_plan;

/* Builds the LANCZOS tables (host, double, as PIL) and allocates the uint8 pyramid
 * scratch on the current device.  NULL on error (see md2_last_error). */
md2_aug_plan* md2_aug_plan_create(const md2_aug_desc* desc);
void md2_aug_plan_destroy(md2_aug_plan* plan);

/*
 * frames: device uint8 (F, B, in_height, in_width, 3), frame-major (frame f of item b
 * at index f*B + b); items: HOST md2_aug_item[B], staged through a pinned ring owned by
 * the plan and uploaded on `stream` (the call does not wait for the GPU; a plan is not
 * thread-safe);
 * color[s] / color_aug[s]: device float32 (F, B, 3, height>>s, width>>s), i.e.
 * inputs[("color", frame_ids[f], s)][b] and inputs[("color_aug", ...)][b].
 */
int md2_aug_run(md2_aug_plan* plan, const uint8_t* frames, const md2_aug_item* items,
                float* const* color, float* const* color_aug, void* stream);
/* ... and (ABI 20) src8, device uint32 (F-1, B, height, width) or NULL: frames 1..F-1
 * (the photometric sources, frame_ids[1:]) at scale 0 as RGBx dwords, byte c = the
 * 8-bit colour whose k/255 is color[0] — md2_tensors.src8, so the hot path's forward
 * does not re-pack them from the fp32 planes. */
int md2_aug_run2(md2_aug_plan* plan, const uint8_t* frames, const md2_aug_item* items,
                 float* const* color, float* const* color_aug, uint32_t* src8, void* stream);

/*
 * Training-mode BatchNorm2d (+ residual add) (+ ReLU) on channels_last activations:
 * relu(bn(x)) and relu(bn(x) + identity) of the ResNet encoders' blocks
 * (torchvision BasicBlock / Bottleneck behind networks/resnet_encoder.py:62-98).
 * x, y, residual and their gradients: (pixels = N*H*W, channels) fp32, or bf16 with
 * MD2_BN_BF16 (NHWC; fp32 arithmetic and statistics);
 * channels a multiple of 4 with channels/4 dividing, or a multiple of, 256.
 * Forward writes y, the batch mean and 1/sqrt(var + eps) (save_*), and updates the
 * running statistics when running_mean/var are given (momentum, unbiased variance,
 * as nn.BatchNorm2d).  workspace: md2_bn_workspace_bytes, no initialisation needed;
 * a backward must not share its workspace with another call in flight.  Three
 * launches each way; deterministic.
 */
#define MD2_BN_RELU     (1u << 0)
#define MD2_BN_RESIDUAL (1u << 1)
#define MD2_BN_BF16     (1u << 2)   /* x, residual, y and their gradients are bf16 (params, stats fp32) */

typedef struct md2_bn_desc {
    int64_t pixels;   /* N*H*W over all groups */
    int32_t channels;
    uint32_t flags;   /* MD2_BN_* */
    float eps, momentum;
    /* groups > 1: the N images form `groups` equal consecutive chunks, each normalised
     * with its own batch statistics, running statistics updated chunk by chunk in
     * order — exactly `groups` separate BatchNorm calls (the pose encoder runs both
     * frame pairs as one batch this way).  save_mean / save_invstd: (groups, C). */
    int32_t groups;
    int32_t reserved;
} md2_bn_desc;

size_t md2_bn_workspace_bytes(const md2_bn_desc* desc);
int md2_bn_fwd(const md2_bn_desc* desc, const void* x, const float* gamma, const float* beta,
               const void* residual, float* running_mean, float* running_var, void* y,
               float* save_mean, float* save_invstd, void* workspace, void* stream);
/* grad_residual = d(loss)/d(residual) (with MD2_BN_RESIDUAL); y is needed with MD2_BN_RELU. */
int md2_bn_bwd(const md2_bn_desc* desc, const void* x, const void* y, const void* grad_y,
               const float* gamma, const float* save_mean, const float* save_invstd,
               void* grad_x, void* grad_residual, float* grad_gamma, float* grad_beta,
               void* workspace, void* stream);
/* md2_bn_bwd with the output gradient given as up to three tensors summed on load
 * (grad_y + grad_y2 + grad_y3; grad_y2 / grad_y3 may be NULL): the output's other
 * consumers (the next block's shortcut, the decoder skip) hand their gradients here
 * instead of autograd adding them in separate passes. */
int md2_bn_bwd_multi(const md2_bn_desc* desc, const void* x, const void* y, const void* grad_y,
                     const void* grad_y2, const void* grad_y3, const float* gamma, const float* save_mean,
                     const float* save_invstd, void* grad_x, void* grad_residual, float* grad_gamma,
                     float* grad_beta, void* workspace, void* stream);
/* ABI 15: the ReLU mask instead of y.  md2_bn_fwd_mask = md2_bn_fwd that also writes
 * relu_mask (MD2_BN_RELU only; NULL = none): one byte per element quad of y, bit i set
 * when element 4q + i of y (as stored: bf16 after rounding) is > 0 — pixels*channels/4
 * bytes.  md2_bn_bwd_mask = md2_bn_bwd_multi gated by that mask instead of reading y
 * (1/16 of y's bytes in fp32): same results, bit for bit. */
int md2_bn_fwd_mask(const md2_bn_desc* desc, const void* x, const float* gamma, const float* beta,
                    const void* residual, float* running_mean, float* running_var, void* y, uint8_t* relu_mask,
                    float* save_mean, float* save_invstd, void* workspace, void* stream);
int md2_bn_bwd_mask(const md2_bn_desc* desc, const void* x, const uint8_t* relu_mask, const void* grad_y,
                    const void* grad_y2, const void* grad_y3, const float* gamma, const float* save_mean,
                    const float* save_invstd, void* grad_x, void* grad_residual, float* grad_gamma,
                    float* grad_beta, void* workspace, void* stream);

/*
 * The ResNet stem's MaxPool2d(3, stride 2, padding 1) on channels_last activations
 * (x: (batch, height, width, channels), channels a multiple of 4; fp32, or bf16 with
 * MD2_POOL_BF16).  idx: one byte per output value, the winning window position 0..8
 * (first maximum in scan order; NaN propagates, as ATen), uint32-packed per 4
 * channels: batch * ho * wo * channels / 4 words.  The backward gathers (no atomics).
 */
#define MD2_POOL_BF16 (1u << 0)

typedef struct md2_pool_desc {
    int32_t batch, channels, height, width;
    uint32_t flags;
    int32_t reserved;
} md2_pool_desc;

int md2_maxpool3s2_fwd(const md2_pool_desc* desc, const void* x, void* y, uint32_t* idx, void* stream);
int md2_maxpool3s2_bwd(const md2_pool_desc* desc, const uint32_t* idx, const void* grad_y, void* grad_x,
                       void* stream);
/* grad_x = the pool's adjoint of grad_y + grad_add (same shape and layout as x; NULL
 * = none): the stem activation also feeds the DepthDecoder skip (resnet_encoder.py:96
 * features[0]), so its two gradients are summed in the gather instead of a separate
 * add pass. */
int md2_maxpool3s2_bwd_add(const md2_pool_desc* desc, const uint32_t* idx, const void* grad_y, const void* grad_add,
                           void* grad_x, void* stream);
/* ... and grad_y2 (NULL = none) a second gradient of the pooled map y, same shape and
 * layout as grad_y, summed into it on load: y feeds both the first BasicBlock's conv1 and
 * its identity shortcut (torchvision BasicBlock.forward, `identity = x`), so autograd
 * would otherwise add the two gradients in a separate pass. (ABI 19) */
int md2_maxpool3s2_bwd_multi(const md2_pool_desc* desc, const uint32_t* idx, const void* grad_y, const void* grad_y2,
                             const void* grad_add, void* grad_x, void* stream);

/*
 * fp32 convolutions as implicit GEMMs on f32 MFMA (csrc/conv.hip): the ResNet
 * encoders' 3x3 / 1x1 convolutions (networks/resnet_encoder.py, torchvision
 * BasicBlock/Bottleneck) and the DepthDecoder's 3x3 convolutions on reflection-padded
 * inputs (networks/depth_decoder.py:50-65 via layers.py:106-136 Conv3x3; the padding
 * is md2_decoder_pad_fwd's, so pad = 0), forward and backward, replacing MIOpen.
 * x (batch, height, width, in_channels) NHWC fp32; weight (out_channels, kernel_h,
 * kernel_w, in_channels) = a channels_last Conv2d weight; y (batch, Ho, Wo,
 * out_channels) NHWC with Ho = (height + 2 pad - kernel_h) / stride + 1.  No bias.
 * Channel counts multiples of 4, pad < kernel, every tensor < 2^29 elements.  Zero
 * padding outside the image.  Deterministic (a K split sums its partials in order);
 * workspace of md2_conv_workspace_bytes (0 = none needed).
 */
#define MD2_CONV_NO_SPLIT  (1u << 1) /* no K split (tests)              */
#define MD2_CONV_TILE_N32  (1u << 2) /* force the 128 x 32 tile (tests) */
#define MD2_CONV_TILE_N64  (1u << 3) /* force the 128 x 64 tile         */
#define MD2_CONV_TILE_N128 (1u << 4) /* force the 128 x 128 tile        */
#define MD2_CONV_X6        (1u << 5) /* split-bf16 (3 planes, 6 products) f32-class MFMA path */
#define MD2_CONV_BM256     (1u << 6) /* x6 forward / input grad: 256 x 128 tiles (N > 64)     */
#define MD2_CONV_PRESPLIT  (1u << 7) /* x6: `weight` holds md2_conv_split_weights planes      */
#define MD2_CONV_PATCH     (1u << 8) /* x6 3x3 stride 1: fwd / dgrad (GEMM channels % 32) with
                                        the input patch of a pixel rectangle staged once for
                                        all nine taps (conv_x6p_kernel); the weight gradient
                                        with three input rows per 32-pixel segment staged
                                        once for the nine taps (conv_x6pw_kernel)           */
#define MD2_CONV_S2_ONE    (1u << 9) /* x6 stride-2 input gradient: the four parity classes
                                        in one launch, no K split                           */
#define MD2_CONV_WS        (1u << 10) /* x6 forward / stride-1 input gradient, 128-wide tiles: the
                                         warp-specialised kernel (4 MFMA + 4 staging waves) */
#define MD2_CONV_BF16      (1u << 11) /* ABI 22: a bf16 autocast convolution (config C5): x, y,
                                         grad_y, grad_x are bf16 NHWC; `weight` of md2_conv_fwd /
                                         md2_conv_dgrad is ONE bf16 plane of
                                         md2_conv_bf16_weights; grad_weight stays fp32, holding
                                         bf16-rounded values (the autocast cast's backward).
                                         f32 accumulation, output rounded to nearest even,
                                         deterministic (fixed-order K split).  fwd: in_channels
                                         % 8; dgrad: stride 1, out_channels % 8 */

typedef struct md2_conv_desc {
    int32_t batch, height, width, in_channels; /* input */
    int32_t out_channels, kernel_h, kernel_w, stride, pad;
    uint32_t flags;                            /* MD2_CONV_* */
} md2_conv_desc;

size_t md2_conv_workspace_bytes(const md2_conv_desc* desc);
/* The split-bf16 weight planes of md2_conv_fwd / md2_conv_dgrad with MD2_CONV_X6 in
 * one pass: planes_fwd [3][Co][KH*KW][Ci] bf16 and (nullable) planes_dgrad
 * [3][Ci][KH*KW][Co] (taps flipped); pass them as `weight` with MD2_CONV_PRESPLIT.
 * Channels must be multiples of 8. */
int md2_conv_split_weights(const md2_conv_desc* desc, const float* weight, void* planes_fwd, void* planes_dgrad,
                           void* stream);
/* Every conv weight of a training step split in ONE launch (the per-convolution
 * md2_conv_split_weights launches of the forward, ~80 tiny kernels per step, become one
 * ~10k-block grid): `table` is a DEVICE array of `n` entries; entry e covers grid blocks
 * [block0, block0 + ceil(ci/32) * ceil(co/32) * kt) in ascending order, and
 * `total_blocks` is the last entry's end.  Same planes as md2_conv_split_weights
 * (planes_dgrad nullable per entry).  Graph-capturable (no host sync). */
typedef struct md2_wsplit_entry {
    const float* weight;        /* (co, kt, ci) channels_last conv weight        */
    void* planes_fwd;           /* [3][co][kt][ci] bf16                           */
    void* planes_dgrad;         /* [3][ci][kt][co] bf16, taps flipped, or NULL    */
    int32_t co, kt, ci;         /* out channels, kernel_h * kernel_w, in channels */
    int32_t block0;             /* first grid block of this entry                 */
    void* planes_col;           /* [3][kt][ci][co] bf16 (taps not flipped), or NULL: the
                                   weight as the 1x1 GEMM operand of a strided input
                                   gradient's column form (md2_conv_col2im; ABI 19) */
} md2_wsplit_entry;
int md2_conv_split_weights_multi(const md2_wsplit_entry* table, int n, int total_blocks, void* stream);
/* MD2_CONV_BF16 operands (ABI 22): the fp32 weight rounded to bf16 (nearest even) in the
 * forward layout w_fwd [Co][KH*KW][Ci] and (nullable) the input gradient's w_dgrad
 * [Ci][KH*KW][Co] with the taps flipped — what autocast's bf16 cast of the weight feeds a
 * bf16 convolution, in the two GEMM layouts.  The _multi form converts a whole table of
 * weights in one launch (md2_wsplit_entry: planes_fwd / planes_dgrad receive the one
 * plane each, planes_col unused). */
int md2_conv_bf16_weights(const md2_conv_desc* desc, const float* weight, void* w_fwd, void* w_dgrad, void* stream);
int md2_conv_bf16_weights_multi(const md2_wsplit_entry* table, int n, int total_blocks, void* stream);
int md2_conv_fwd(const md2_conv_desc* desc, const float* x, const float* weight, float* y, void* workspace,
                 void* stream);
/* grad_x (batch, height, width, in_channels) from grad_y (batch, Ho, Wo, out_channels):
 * stride 1 (a "full" convolution with the flipped, transposed weight), or stride 2 with
 * MD2_CONV_X6 and >= 32 out_channels (four output-parity classes, each a stride-1 GEMM
 * over its taps, scattered into grad_x) */
int md2_conv_dgrad(const md2_conv_desc* desc, const float* grad_y, const float* weight, float* grad_x,
                   void* workspace, void* stream);
/* The gather half of a strided input gradient computed as one GEMM: cols (batch, Ho, Wo,
 * kernel_h, kernel_w, in_channels) — grad_y times the weight as [out][(kh, kw, ci)], a 1x1
 * md2_conv_fwd with kernel_h*kernel_w*in_channels outputs — summed into grad_x (batch,
 * height, width, in_channels): each pixel gathers its taps in (kh, kw) order, written
 * (not accumulated).  in_channels % 4; replaces the parity-class launches of a stride-2
 * md2_conv_dgrad (MIOpen's backward-data convolution, networks/resnet_encoder.py). */
int md2_conv_col2im(const md2_conv_desc* desc, const float* cols, float* grad_x, void* stream);
/* grad_weight (out_channels, kernel_h, kernel_w, in_channels) = channels_last layout */
int md2_conv_wgrad(const md2_conv_desc* desc, const float* x, const float* grad_y, float* grad_weight,
                   void* workspace, void* stream);
/* Direct 3x3 stride-1 convolution on the f32 VALU (csrc/direct.hip) for the
 * DepthDecoder's 16-output-channel layers (networks/depth_decoder.py:50-65:
 * upconv(0,0) 32->16, upconv(0,1) 16->16) and their input gradients: y (batch, Ho, Wo,
 * out_channels) = x (batch, height, width, in_channels) correlated with
 * wk [9][in_channels][out_channels] (tap-major; for the input gradient: the flipped
 * weight with its channel roles swapped, pad = 2 - the forward's pad), zero padding
 * `pad` (0..2), Ho = height + 2 pad - 2.  (in, out) channels (16,16), (32,16) or
 * (16,32); kernel 3x3, stride 1; desc flags unused.  One thread per output pixel,
 * exact f32 FMA chains. */
int md2_conv_direct(const md2_conv_desc* desc, const float* x, const float* wk, float* y, void* stream);
/* Weight gradient of the same layers on the f32 VALU: grad_weight (out_channels, 3, 3,
 * in_channels) = sum over output pixels of grad_y x the input's tap; (in, out) channels
 * (16,16) or (32,16), stride 1, pad 0..2.  Per-block partial rows in `workspace`
 * (md2_conv_wgrad_direct_workspace_bytes), summed in block order (deterministic). */
size_t md2_conv_wgrad_direct_workspace_bytes(const md2_conv_desc* desc);
int md2_conv_wgrad_direct(const md2_conv_desc* desc, const float* x, const float* grad_y, float* grad_weight,
                          void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MD2HOT_H */
