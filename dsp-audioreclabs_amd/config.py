"""Configuration constants of the reference (config.py:29-70), for drop-in callers.

Unlike the reference, importing this module has no side effects: RESULTS_DIR is created by the
experiment runner when it writes, not at import (the reference's config.py:25-26 makedirs).
"""
import os

BASE_DIR = os.path.dirname(os.path.abspath(__file__))
DATASET_TYPE = os.environ.get('DATASET_TYPE', 'name')
DATASET_PATHS = {
    'name': os.path.join(os.path.expanduser('~'), 'Downloads', 'speech_data_name'),
    'number': os.path.join(os.path.expanduser('~'), 'Downloads', 'speech_data_number'),
}
DATA_DIR = os.environ.get('SPEECH_DATA_DIR', DATASET_PATHS.get(DATASET_TYPE, DATASET_PATHS['name']))
RESULTS_DIR = os.path.join(BASE_DIR, 'results')

# audio / framing (config.py:29-40)
SAMPLE_RATE = 44100
NORMALIZE = True
FRAME_LENGTH_MS = 25
FRAME_SHIFT_MS = 10
FRAME_LENGTH = int(SAMPLE_RATE * FRAME_LENGTH_MS / 1000)   # 1102
FRAME_SHIFT = int(SAMPLE_RATE * FRAME_SHIFT_MS / 1000)     # 441
# Frame sizes in samples, overriding the ms values above: BASELINE.json configs[0] quotes the
# reference's CPU run at 1024 / 512 samples, which no integer-ms setting of config.py:35-40 gives
# (int(44100 * ms / 1000)).  Environment DSP_FRAME_LENGTH / DSP_FRAME_SHIFT, or
# run.py --frame-length / --frame-shift.
FRAME_LENGTH = int(os.environ.get('DSP_FRAME_LENGTH', FRAME_LENGTH))
FRAME_SHIFT = int(os.environ.get('DSP_FRAME_SHIFT', FRAME_SHIFT))

# endpoint detection (config.py:43-45)
ENERGY_HIGH_RATIO = 0.5
ENERGY_LOW_RATIO = 0.1
ZCR_THRESHOLD_RATIO = 1.5

WINDOW_TYPES = ['rectangular', 'hamming', 'hanning']
FEATURE_STATS = ['mean', 'std', 'max', 'min', 'median']

# classifiers (config.py:55-66)
KNN_N_NEIGHBORS = 3
SVM_C = 1.0
SVM_KERNEL = 'rbf'
MLP_HIDDEN_LAYERS = [64, 64, 32]
MLP_LEARNING_RATE = 0.005
MLP_EPOCHS = 1000
MLP_BATCH_SIZE = 108

TEST_SIZE = 0.2
RANDOM_SEED = 42
FIGURE_DPI = 150
FIGURE_SIZE = (12, 8)
