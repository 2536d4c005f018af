# round-4 call 29: the other model families at HEAD (LeNet-5, word2vec, char-LSTM; scripts/bench_models.py)
set -u
STEPS="models" bash scripts/gpu_session.sh
