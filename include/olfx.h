/*
 * include/olfx.h -- C-ABI of the MI355X bulk audio-effect engine (libolfx.so).
 *
 * One engine = one effect kind x N independent instances on one GPU.  Every call processes a
 * block of frames for ALL instances at once on a HIP stream; per-instance parameters and note
 * events are applied at the next block boundary (the JUCE-host pattern, reference
 * modules/juce/host/host.cpp:646-653).  No torch types, plain pointers and sizes only.
 *
 * What each entry point replaces in the reference (/root/reference):
 *   olfx_create / olfx_destroy  <- DattorroVerb_create / _delete (libs/dattorro-verb/verb.h:5-8,
 *                                  verb.cpp:225-251); fxlib XxxFx::Init(sr) (modules/fxlib/Fx.h:183,
 *                                  :290); SynthVoice::Init(sr) (modules/synthlib/SynthVoice.h:31-39);
 *                                  README ChorusEffect::init(sr) (README.md:117-127)
 *   olfx_set_params             <- DattorroVerb_set* (verb.h:10-16, verb.cpp:137-170);
 *                                  ChorusEffect::setDepth/setRate (README.md:120-121) and the RNBO
 *                                  chorus params (modules/rnbo/patcher/mono-chorus.rnbopat:431-4353);
 *                                  SynthVoice::UpdateConfig/Update (SynthVoice.h:55-98)
 *   olfx_note_events            <- SynthVoice::NoteOn/NoteOff (SynthVoice.h:245-256)
 *   olfx_process                <- the per-frame loops DattorroVerb_process + getLeft/getRight
 *                                  (verb.cpp:258-325), ReverbFx glue (modules/fxlib/ReverbFx.cpp:11-27),
 *                                  ChorusEffect::process(sample) (README.md:124), SynthVoice::Process
 *                                  (SynthVoice.h:41-53) -- batched: n_frames x n_inst per call
 *   olfx_mix_config / olfx_mix  <- Polyvoice::Process (modules/synthlib/Polyvoice.h:28-33) and
 *                                  VoiceMap::Process (VoiceMap.h:64-73): voices added into one
 *                                  frame, voice by voice
 *   olfx_last_error             <- (reference has none: void returns / NULL, verb.cpp:89-90,227)
 *
 * Audio layout (both host and device pointers accepted, see OLFX_IO_*):
 *   in  : [in_channels ][n_frames][n_inst]  float32, instance index fastest
 *   out : [out_channels][n_frames][n_inst]  float32
 * Channel counts per kind are given by olfx_kind_info().
 *
 * Errors: every function returns 0 on success or a negative OLFX_E_* code; no C++ exception
 * crosses this boundary.  An engine is not re-entrant: one host thread drives one engine.
 */
#ifndef OLFX_H
#define OLFX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OLFX_ABI_VERSION 2

/* ---- status codes ---- */
enum {
    OLFX_OK          = 0,
    OLFX_E_ARG       = -1,   /* bad argument (null, out of range, wrong size) */
    OLFX_E_NOMEM     = -2,   /* host or device allocation failed */
    OLFX_E_HIP       = -3,   /* a HIP runtime call failed; see olfx_last_error */
    OLFX_E_NODEVICE  = -4,   /* no GPU / device index invalid */
    OLFX_E_KIND      = -5,   /* unknown effect kind */
    OLFX_E_STATE     = -6    /* call not valid in the engine's current state */
};

/* ---- effect kinds ---- */
enum {
    OLFX_KIND_DATTORRO   = 1,  /* libs/dattorro-verb: stereo in -> (l+r)/2 -> stereo out (ReverbFx.cpp:11-27),
                                  or mono in (verb.h:19) */
    OLFX_KIND_CHORUS     = 2,  /* RNBO stereo-chorus (mono-chorus x2, shared params) */
    OLFX_KIND_PITCHSHIFT = 3,  /* gen~ pitchshift, stereo */
    OLFX_KIND_VOICE      = 4,  /* synthlib SynthVoice: polyBLEP saw -> SVF LP (env cutoff) -> amp env; mono out */
    OLFX_KIND_CHAIN      = 5,  /* fused chorus -> pitch-shift -> dattorro, stereo */
    OLFX_KIND_FXRACK     = 6,  /* fxlib ol::fx::FxRack<2>: delay -> reverb -> filter -> master (Fx.h:398-492) */
    OLFX_KIND_VOICE_MOOG = 7   /* SynthVoice(OscillatorSoundSource, MoogFilter): the Daisy synth firmware voice
                                  (ol_daisy/app/synth/main.cpp:49-52); daisysp::LadderFilter LP24 in place of the
                                  SVF (Filter.h:35-63).  Same OLFX_VC_* parameters (FILTER_DRIVE is ignored:
                                  MoogFilter::SetDrive is a no-op), note events and control changes. */
};

/* ---- parameters (field index, value is what the reference setter takes) ---- */
/* Dattorro: verb.h:10-16 */
enum {
    OLFX_DT_PREDELAY = 0,        /* setPreDelay: [0,1] x 4800 samples, per instance */
    OLFX_DT_PREFILTER,           /* setPreFilter */
    OLFX_DT_INPUT_DIFFUSION1,    /* setInputDiffusion1 */
    OLFX_DT_INPUT_DIFFUSION2,    /* setInputDiffusion2 */
    OLFX_DT_DECAY_DIFFUSION,     /* setDecayDiffusion */
    OLFX_DT_DECAY,               /* setDecay (also derives decay diffusion 2, verb.cpp:164) */
    OLFX_DT_DAMPING,             /* setDamping */
    OLFX_DT_NPARAMS
};
/* Chorus (RNBO params, clamped to @min/@max like RNBO; mono-chorus.rnbopat line of each param) */
enum {
    OLFX_CH_PITCH = 0,   /* [0,3]      default 0    :431   pitch-shifter phasor rate, Hz */
    OLFX_CH_MIX,         /* [0,1]      default 0.5  :1772 */
    OLFX_CH_Q,           /* [0,1]      default 0.5  :2226  lores~ resonance */
    OLFX_CH_CUTOFF,      /* [0,1]      default 0.3  :2660  -> 300..15000 Hz (:2242) */
    OLFX_CH_PHASE,       /* [0,1]      default 1    :3420  cycle~ phase offset */
    OLFX_CH_DEPTH,       /* [0.08,1]   default 0.5  :3854  -> 1..12 ms (:3436) */
    OLFX_CH_RATE,        /* [0.01,1]   default 0.2  :4353  -> 0.01..0.5 Hz (:3935) */
    OLFX_CH_WINDOW,      /* [4,10] ms  default 10   pitchshift.gendsp "Param window" */
    OLFX_CH_NPARAMS
};
/* Pitch-shift stage (gen~ pitchshift.gendsp) */
enum {
    OLFX_PS_SHIFT = 0,   /* [0,3] Hz phasor rate (inlet 2 of pitchshift.gendsp) */
    OLFX_PS_WINDOW,      /* [4,10] ms */
    OLFX_PS_NPARAMS
};
/* Voice: Voice::Config field order (modules/synthlib/Voice.h:14-31) */
enum {
    OLFX_VC_FILTER_CUTOFF = 0, OLFX_VC_FILTER_RESONANCE, OLFX_VC_FILTER_DRIVE, OLFX_VC_FILTER_ENV_AMOUNT,
    OLFX_VC_FILTER_ATTACK, OLFX_VC_FILTER_ATTACK_SHAPE, OLFX_VC_FILTER_DECAY, OLFX_VC_FILTER_SUSTAIN,
    OLFX_VC_FILTER_RELEASE, OLFX_VC_AMP_ENV_AMOUNT, OLFX_VC_AMP_ATTACK, OLFX_VC_AMP_ATTACK_SHAPE,
    OLFX_VC_AMP_DECAY, OLFX_VC_AMP_SUSTAIN, OLFX_VC_AMP_RELEASE, OLFX_VC_PORTAMENTO,
    OLFX_VC_NPARAMS
};
/* Effect rack: ol::fx::FxRack<2> members (modules/fxlib/Fx.h; defaults in brackets) */
enum {
    OLFX_FR_DELAY_TIME = 0,      /* DelayFx time [0,1] -> 0..48000 samples            [0.5]   Fx.h:172,214 */
    OLFX_FR_DELAY_FEEDBACK,      /* DelayFx feedback                                   [0.5]   Fx.h:173 */
    OLFX_FR_DELAY_BALANCE,       /* DelayFx wet/dry                                    [0.33]  Fx.h:174 */
    OLFX_FR_DELAY_CUTOFF,        /* DelayFx filter_ cutoff, Hz              [scale(64,0,127,0,20000)] :188 */
    OLFX_FR_DELAY_RESONANCE,     /* DelayFx filter_ resonance [0,1]            [scale(24,0,127,0,1)] :189 */
    OLFX_FR_REVERB_BALANCE,      /* ReverbFx balance (over the ReverbSc stub)   [0.1]   Fx.h:282 */
    OLFX_FR_FILTER_CUTOFF,       /* FxRack filter1 cutoff, Hz                  [20000]  Fx.h:75 */
    OLFX_FR_FILTER_RESONANCE,    /* [0] */
    OLFX_FR_FILTER_DRIVE,        /* [0] */
    OLFX_FR_FILTER_TYPE,         /* 0 low, 1 band, 2 high, 3 notch, 4 peak      [0]     Fx.h:67-73 */
    OLFX_FR_MASTER_VOLUME,       /* [0.8] Fx.h:405 */
    OLFX_FR_TOPOLOGY,            /* [0] 0: FxRack<2>::Process (Fx.h:432-440): delay -> reverb -> filter1 into the
                                    zeroed buf_c -> x master (output channel 1 is 0).
                                    1: the Daisy synth firmware's audio callback (ol_daisy/app/synth/main.cpp:
                                    78-86): DelayFx<1> on channel 0 -> stereo[0] = stereo[1] -> ReverbFx<2>
                                    -> FilterFx<2> in place (channel 1 keeps the reverb's output), no master
                                    volume (MASTER_VOLUME ignored).  Input: the mono signal in channel 0.
                                    Controls (olfx_control) follow the firmware too (main.cpp:201-207): the
                                    voice-filter CCs 41-44 drive FILTER_*, CCs 45-48 and 7 are ignored.
                                    2, 3, 4: one component alone, as the firmware's objects (main.cpp:82-85):
                                    2 DelayFx<2>::Process (Fx.h:193-206; DELAY_* fields; channel 0 filtered
                                      by its filter_, channel 1 not; DelayFx<1> = channel 0);
                                    3 ReverbFx<2>::Process over the ReverbSc stub (Fx.h:293-299; REVERB_BALANCE):
                                      per channel 0.8 in balance + in (1 - balance);
                                    4 FilterFx<2>::Process (Fx.h:88-108; FILTER_*): the Svf on channel 0, and
                                      channel 1 passes through (the reference leaves frame_out[1] unwritten:
                                      in place, as the firmware calls it, that is channel 1 of the input).
                                    olfx_control gives each its own controls only (DelayFx 35-39, ReverbFx 34,
                                    FilterFx 41-44).  One engine may mix every topology. */
    OLFX_FR_NPARAMS
};
/* Chain: chorus params, then pitch-shift params, then dattorro params */
#define OLFX_CN_CHORUS0   0
#define OLFX_CN_PITCH0    (OLFX_CH_NPARAMS)
#define OLFX_CN_VERB0     (OLFX_CH_NPARAMS + OLFX_PS_NPARAMS)
#define OLFX_CN_NPARAMS   (OLFX_CH_NPARAMS + OLFX_PS_NPARAMS + OLFX_DT_NPARAMS)

/* ---- note events (voices) ----
   The ol::synth::Voice calls that change a voice's gate or pitch (Voice.h:33-57), as SynthVoice
   implements them (SynthVoice.h:231-268):
     NOTE_ON        NoteOn(note, vel)  = GateOn + freq_ = mtof(note) + Retrigger(true) on both envelopes
     NOTE_OFF       NoteOff(note, vel) = GateOff
     GATE_ON        GateOn()           = gate = true (the envelopes see the rising edge, no retrigger)
     GATE_OFF       GateOff()          = gate = false
     SET_FREQUENCY  SetFrequency(hz)   = freq_ = hz (olfx_voice_event.value; olfx_voice_events only) */
enum { OLFX_EV_NOTE_OFF = 0, OLFX_EV_NOTE_ON = 1, OLFX_EV_GATE_ON = 2, OLFX_EV_GATE_OFF = 3,
       OLFX_EV_SET_FREQUENCY = 4 };
typedef struct olfx_event {
    uint32_t inst;      /* instance index */
    uint8_t  type;      /* OLFX_EV_* (not SET_FREQUENCY) */
    uint8_t  note;      /* MIDI note (NoteOn: freq = mtof(note)) */
    uint8_t  velocity;  /* unused by SynthVoice (SynthVoice.h:245) */
    uint8_t  pad;
} olfx_event;
typedef struct olfx_voice_event {
    uint32_t inst;      /* instance index */
    uint8_t  type;      /* OLFX_EV_* */
    uint8_t  note;      /* NOTE_ON: MIDI note */
    uint8_t  velocity;  /* unused by SynthVoice */
    uint8_t  pad;
    float    value;     /* SET_FREQUENCY: Hz (finite); else unused */
} olfx_voice_event;

/* ---- control changes (MIDI CC / hardware controls; corelib/cc_map.h numbers) ----
   The reference's UpdateMidiControl(control, 0..127) / UpdateHardwareControl(control, float)
   mapped to one parameter field, per kind:
     OLFX_KIND_VOICE : SynthVoice::UpdateMidiControl / UpdateHardwareControl (SynthVoice.h:100-229)
     OLFX_KIND_FXRACK: FxRack::UpdateMidiControl / UpdateHardwareControl (Fx.h:451-489) and the
                       DelayFx / ReverbFx / FilterFx handlers it forwards to (Fx.h:116-163, 218-267, 313-391);
                       olfx_control_map gives topology 0's mapping, olfx_control uses each instance's
                       topology (OLFX_FR_TOPOLOGY 1: the firmware's direct FilterFx routing)
   Controls the reference ignores for a kind (its `default: update = false`) are skipped. */
enum { OLFX_CTL_MIDI = 0, OLFX_CTL_HARDWARE = 1 };
#define OLFX_IGNORED 1                 /* olfx_control_map: the reference ignores this control */
#define OLFX_FIELD_UPDATE_ONLY 0xFFFFFFFFu   /* handled control that sets no modelled field (Update() only) */
typedef struct olfx_control_event {
    uint32_t inst;
    uint8_t  control;   /* CC number, corelib/cc_map.h */
    uint8_t  source;    /* OLFX_CTL_MIDI (value 0..127) or OLFX_CTL_HARDWARE (value as given) */
    uint16_t pad;
    float    value;
} olfx_control_event;

/* ---- I/O flags ---- */
enum {
    OLFX_IO_DEVICE = 0,  /* in/out are device pointers (no copies; the fast path) */
    OLFX_IO_HOST   = 1   /* in/out are host pointers: staged through pinned buffers, PCIe-inclusive */
};

typedef struct olfx_engine olfx_engine;

typedef struct olfx_kind_info {
    int      kind;
    uint32_t n_params;
    uint32_t in_channels;       /* channels olfx_process reads */
    uint32_t out_channels;      /* channels olfx_process writes */
    uint64_t state_bytes_per_instance;   /* device state (rings + scalars + params); a reverb
                                            engine of 2 x 64 x CUs instances or more whose
                                            pre-delays come to differ adds 32 KB per instance (a
                                            copy of the pre-delay ring while its layout changes,
                                            DESIGN.md section 4), allocated at the first such
                                            block, kept until destroy */
} olfx_kind_info;

int olfx_abi_version(void);
int olfx_kind_info_get(int kind, float sample_rate, olfx_kind_info *info);

/* Create an engine of `kind` with n_inst instances on HIP device `device`.  All instances start
   in the reference's freshly-created state (zeroed rings, default parameters).
   block = the frames per olfx_process call the caller intends (any multiple of 4 is accepted). */
int olfx_create(int kind, int device, uint32_t n_inst, float sample_rate, uint32_t block,
                olfx_engine **out);
int olfx_destroy(olfx_engine *e);

/* Zero all state and restore defaults (== destroy + create, without reallocating).  Like
   olfx_destroy and olfx_sync it waits for THIS engine's queued work only (the stream of its latest
   olfx_process / olfx_mix, its own streams, its control packets), never for the whole device:
   other engines and the host's own kernels keep running.  The caller keeps the stream it passed
   last alive until then (and until the next olfx_process / olfx_mix on another stream, which the
   engine orders after its previous launch itself: switching streams between calls needs no event
   from the caller; the caller's own buffers stay the caller's to order). */
int olfx_reset(olfx_engine *e);

/* Set parameters of instances [first, first+count): `values` is field-major
   [n_fields][count] for fields [field0, field0+n_fields).  Host pointer.  Applied at the start
   of the next olfx_process. */
int olfx_set_params(olfx_engine *e, uint32_t first, uint32_t count, uint32_t field0,
                    uint32_t n_fields, const float *values);
/* Convenience: one field of one instance. */
int olfx_set_param(olfx_engine *e, uint32_t inst, uint32_t field, float value);
/* One field of `count` scattered instances: inst[k] gets values[k] (the per-instance setter called
   on each, e.g. one MIDI CC fanned out to many objects).  Validated first: a rejected call changes
   nothing.  Applied at the start of the next olfx_process, like every parameter change; the
   engine re-derives and uploads the coefficients of changed instances only, asynchronously. */
int olfx_set_param_list(olfx_engine *e, uint32_t field, const uint32_t *inst, const float *values,
                        uint32_t count);
/* A member value without Update(): the state the reference's setters leave when they are called
   BEFORE Init (the Daisy firmware configures its voices that way, ol_daisy/app/synth/main.cpp:114-128
   then :149).  For voices, SynthVoice::Init resets the components to DaisySP's defaults, while
   Process keeps reading the members filter_cutoff, filter_env_amount, amp_env_amount and Init hands
   portamento_htime to the Port (SynthVoice.h:31-53): the field is stored without the Update() that
   olfx_set_params implies.  For the other kinds it is olfx_set_param. */
int olfx_set_member(olfx_engine *e, uint32_t inst, uint32_t field, float value);
/* Read back the current (host shadow) value of one parameter. */
int olfx_get_param(olfx_engine *e, uint32_t inst, uint32_t field, float *value);

/* Map one control change to (field, value) exactly as the reference handler scales it
   (ol::core::scale, corelib/ol_corelib.h:31-44).  Returns OLFX_OK, OLFX_IGNORED, or an error.
   Pure host function: no engine, no device. */
int olfx_control_map(int kind, uint8_t control, int source, float value, uint32_t *field, float *param_value);
/* Apply control changes in order (each: the mapped olfx_set_param; ignored controls skipped).
   Replaces UpdateMidiControl / UpdateHardwareControl per instance. */
int olfx_control(olfx_engine *e, const olfx_control_event *ev, uint32_t n);

/* Queue note events (voices); applied in order at the start of the next olfx_process. */
int olfx_note_events(olfx_engine *e, const olfx_event *ev, uint32_t n);
/* The same queue with SET_FREQUENCY (Voice::SetFrequency, SynthVoice.h:264-267) as well. */
int olfx_voice_events(olfx_engine *e, const olfx_voice_event *ev, uint32_t n);

/* Update() of instances [first, first + count) with their current parameters (SynthVoice.h:66-98,
   Fx.h Update()): for voices, the first Update() ends SynthVoice::Init's component defaults
   (olfx_set_params and olfx_control imply it).  Applied at the next olfx_process. */
int olfx_update(olfx_engine *e, uint32_t first, uint32_t count);

/* Process n_frames (multiple of 4) for all instances.  `stream` is a hipStream_t; NULL is the
   HIP default (null) stream, as everywhere in HIP; olfx_stream(e) is the engine's own stream.
   With OLFX_IO_DEVICE the call is asynchronous on that stream. */
int olfx_process(olfx_engine *e, const float *in, float *out, uint32_t n_frames, int io_flags,
                 void *stream);

/* ---- voice buses (voice engines): the Polyvoice / VoiceMap sums ----
   Polyvoice::Process (modules/synthlib/Polyvoice.h:28-33) and VoiceMap::Process (VoiceMap.h:64-73)
   add their voices' samples into the caller's frame one voice at a time (`*frame_out += sample`).
   A bus is such a list.  olfx_mix_config sets the buses (host arrays, copied): bus b adds the
   voices order[offsets[b] .. offsets[b+1]) in that order; offsets has n_buses + 1 entries and
   starts at 0.  A voice may appear at most once over all buses (listed twice, the reference would
   run it twice per frame); n_buses = 0 removes the buses.
   olfx_mix adds, for every frame f and bus b, the bus's voice samples voice_out[f][v] into
   bus_out[f][b] in list order: the reference's float adds, bit for bit.  voice_out is
   [n_frames][n_inst] (this engine's olfx_process output); bus_out is [n_frames][n_buses] and is
   accumulated into (the reference's caller zeroes its frame).  Both host (OLFX_IO_HOST) or both
   device pointers (OLFX_IO_DEVICE: asynchronous on `stream`, as olfx_process). */
int olfx_mix_config(olfx_engine *e, uint32_t n_buses, const uint32_t *offsets, const uint32_t *order);
int olfx_mix(olfx_engine *e, const float *voice_out, float *bus_out, uint32_t n_frames, int io_flags,
             void *stream);

/* Block until all work queued by this engine is done (engine-scoped, see olfx_reset). */
int olfx_sync(olfx_engine *e);
/* The engine's own non-blocking hipStream_t (valid until olfx_destroy). */
void *olfx_stream(const olfx_engine *e);

/* Engine facts. */
uint32_t olfx_num_instances(const olfx_engine *e);
int      olfx_kind(const olfx_engine *e);
uint64_t olfx_frames_processed(const olfx_engine *e);   /* per instance, since create/reset */
uint32_t olfx_num_buses(const olfx_engine *e);          /* voice buses (olfx_mix_config) */
/* Algorithmic ("compulsory") HBM bytes per instance-frame of the dominant kernel, the figure
   bench.py's roofline uses. */
double   olfx_algorithmic_bytes_per_frame(const olfx_engine *e);
/* The read share of the same figure: tap reads of data older than the block plus the input (the
   north star's "HBM-read roofline", SURVEY.md section 8d "read-only variant"). */
double   olfx_algorithmic_read_bytes_per_frame(const olfx_engine *e);
const char *olfx_kernel_name(const olfx_engine *e);
const char *olfx_last_error(const olfx_engine *e);   /* e may be NULL: last global error */

#ifdef __cplusplus
}
#endif
#endif /* OLFX_H */
