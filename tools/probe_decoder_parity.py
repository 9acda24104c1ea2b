import os, sys
sys.path[:0]=['/root/repo','/root/repo/enhance-cb-whisper_amd','/root/repo/tests']
import numpy as np, torch
from cbw import synth
import test_gpu_decoder as T
gd='/root/repo/tests/golden'
g=np.load(os.path.join(gd,'decoder_micro.npz'))
from cbw.generate import beam_search
from test_oracle_golden import suppression_bias
eng=T.decoder_engine()
prefix=g["beam_prefix"].tolist(); V=synth.WHISPER_DECODERS["micro"][0]
nb=suppression_bias(V, g["suppress"].tolist(), len(prefix)); cache={}
def bias_at(pos):
    b=nb(pos); k=id(b)
    if k not in cache: cache[k]=torch.from_numpy(b).float().to(eng.device)
    return cache[k]
eng.start(torch.from_numpy(g["enc_out"])[None], rows=5)
out=beam_search(eng.step_fn(10,bias_at), prefix, 5, 50257, len(prefix)+24, decoder_prompt_len=len(prefix))
ref=g["beam_out"].tolist()
print("beam: len out", len(out), "len ref", len(ref), "prefix", len(prefix), "equal", out==ref)
n=next((i for i,(a,b) in enumerate(zip(out,ref)) if a!=b), min(len(out),len(ref))); print("n_same", n)
from model.pba_whisper import PBAWhisper
gl=np.load(os.path.join(gd,'longform_micro.npz'))
w=PBAWhisper(synth.WHISPER_CONFIGS["micro"], synth.WHISPER_DECODERS["micro"], T.micro_whisper_sd(), suppress_tokens=[1,2,7], max_initial_timestamp_index=50)
feats=torch.from_numpy(gl["features"])[None].to(w.device)
res=w.generate(input_features=feats, task="transcribe", language="en", return_timestamps=True, condition_on_prev_tokens=False, return_segments=True, num_beams=1)
seq=res["sequences"][0].tolist(); r=gl["sequence"].tolist()
n=next((i for i,(a,b) in enumerate(zip(seq,r)) if a!=b), min(len(seq),len(r)))
print("longform: len", len(seq), len(r), "n_same", n, "equal", seq==r)
