import numpy as np, torch, sys
sys.path.insert(0, '/root/repo')
from oracle import whisper_np as W
from whisper_context_biasing_amd.config import get_dims
from whisper_context_biasing_amd.model import WhisperCB
from whisper_context_biasing_amd.synth import synth_batch
from whisper_context_biasing_amd.weights import make_weights
dims = get_dims("micro"); sd = make_weights(dims, seed=0, recipe="diverse")
om = W.OracleModel.from_dims(dims, sd); mel = W.log_mel(synth_batch(2), dims.n_mel); enc = om.encode(mel)
prompt = [50361, 100, 200, 300]
ref = om.generate(mel, enc=enc, max_length=10, prefix=prompt + [dims.decoder_start_token_id], min_new_tokens=10)
print("oracle", ref.tolist())
for trial in range(2):
    m = WhisperCB.from_state_dict(dims, sd, dtype="f32")
    if trial == 1:
        g = np.load('/root/repo/tests/golden/model_micro_diverse_s0.npz')
        m.forward(torch.from_numpy(mel), decoder_input_ids=torch.from_numpy(g["tf_decoder_input_ids"]))
    for ug in (False, True):
        ids = m.generate(torch.from_numpy(mel), max_length=10, prompt_ids=prompt, min_new_tokens=10, use_graph=ug).cpu().numpy()
        print(trial, ug, ids.tolist(), np.array_equal(ids, ref))
