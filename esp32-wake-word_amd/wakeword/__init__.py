"""wakeword -- MI355X-native wake-word inference (MFCC front-end + xiaoa CNN).

Drop-in for the reference's Python surface (ml_models/src/wakeModel.py,
ml_models/src/extract_mfcc.py, the xiaoa.onnx artefact); every compute call
runs a hand-written gfx950 HIP kernel from libwakeword.so.
"""
from ._lib import WakewordError, lib  # noqa: F401
from .api import (EspMfcc, KWSModel, detect, extract_mfcc, load_onnx, load_wav, mfcc, normalize_mfcc, pack_weights,  # noqa: F401
                  pad_audio, synth_clips)
from .onnx_reader import read_onnx, xiaoa_state_dict  # noqa: F401
from .stream import (DecisionRule, DeviceDetector, FrameDecisionLoop, FrameWindow, StreamingDetector,  # noqa: F401
                     Window, device_cmvn, quantize_frames, record_front)
from .ctc import CTCModel, ctc_state_dict_spec, decode_predictions, pack_state_dict, tokens_to_text  # noqa: F401
from . import wav  # noqa: F401

LightweightKWS = KWSModel
