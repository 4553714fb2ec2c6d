/*
 * tests/cpp/test_ref_standalone.cpp -- include/olfx_ref.hpp on its own, without the reference's
 * headers (TEST INFRASTRUCTURE): the restated ol::synth::Voice / SoundSource are complete, the
 * classes construct as the reference constructs them, and without a GPU the first Process throws
 * OLFX_E_NODEVICE (there is no CPU path).  Exit 0 = as expected.
 */
#include <cstdio>
#include <vector>

#include "olfx_ref.hpp"

int main() {
    ol::synth::SynthVoice v1(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice v2;
    std::vector<ol::synth::Voice *> voices{&v1, &v2};
    int bad = 0;
    if (!v1.moog() || v2.moog()) { std::printf("filter kind not picked from the component\n"); ++bad; }
    struct Lines { int dummy; };
    std::vector<Lines *> lines;
    struct Sc { int dummy; } sc;
    ol::fx::DelayFx<2> delay(lines);
    ol::fx::DaisyVerb<2> dv(sc);
    ol::fx::ReverbFx<2> reverb(dv);
    ol::fx::FilterFx<2> filter;
    ol::fx::FxRack<2> rack(delay, reverb, filter);
    delay.UpdateMidiControl(35, 10);                  // before Init: kept, replayed at Init
    int code = 0;
    try {
        for (ol::synth::Voice *v : voices) v->Init(48000.f);
        ol::synth::Voice::Config cfg{};
        voices[0]->UpdateConfig(cfg);
        voices[0]->NoteOn(60, 100);
        if (voices[0]->Playing() != 60 || !voices[0]->Gate()) { std::printf("Playing/Gate\n"); ++bad; }
        rack.Init(48000.f);
        float out = 0.f;
        voices[0]->Process(&out);                     // the generation's first run: needs a GPU
    } catch (const olfx::Error &e) {
        code = e.code();
        std::printf("%s\n", e.what());
    }
    int kind_code = 0;
    struct OtherSource : ol::synth::SoundSource<1> {
        ol::synth::InitStatus Init(t_sample) override { return ol::synth::Ok; }
        void Process(t_sample *) override {}
        void GateOn() override {}
        void GateOff() override {}
        void SetFreq(t_sample) override {}
    } other;
    try { ol::synth::SynthVoice v3(&other); } catch (const olfx::Error &e) { kind_code = e.code(); }
    if (kind_code != OLFX_E_KIND) { std::printf("foreign SoundSource accepted\n"); ++bad; }
    std::printf("code %d, %d problems\n", code, bad);
    return (code == OLFX_E_NODEVICE && bad == 0) ? 0 : 1;
}
