import os, sys
sys.path[:0] = ['/root/repo', '/root/repo/esp32-wake-word_amd']
REPO = os.environ.get('GRAFT_REPO_ROOT', '/root/repo'); sys.path[:0] = [REPO, REPO + '/esp32-wake-word_amd']
import numpy as np, torch, wakeword
from oracle import wk_oracle as O
m32 = wakeword.load_onnx(REPO + '/tests/golden/xiaoa.onnx')
m16 = wakeword.load_onnx(REPO + '/tests/golden/xiaoa.onnx', precision='bf16')
x = O.synth_clips(5, 0, 2000, 16000)
a = m32.detect(x).reshape(-1).cpu().numpy(); b = m16.detect(x).reshape(-1).cpu().numpy()
print('synth max|d|', np.abs(a - b).max(), 'mean|d|', np.abs(a - b).mean(), 'range', a.min(), a.max())
w = np.load(REPO + '/tests/golden/wavs.npz')
a = m32.detect(w['x_noise']).reshape(-1).cpu().numpy(); b = m16.detect(w['x_noise']).reshape(-1).cpu().numpy()
print('wav', a, b, np.abs(a-b).max())
