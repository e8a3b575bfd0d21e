"""Bisect helper: 2-rank fused BERT on one GPU (gloo); env DP_EXTRA adds CLI flags."""
import os, subprocess, sys, socket, tempfile
sys.path.insert(0, os.getcwd())
from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab
t = tempfile.mkdtemp()
d = os.path.join(t, "bert")
write_bert_shards(d, num_shards=2, per_shard=64, seq_len=64, max_pred=8, vocab_size=1000, split="train")
write_bert_shards(d, num_shards=1, per_shard=8, seq_len=64, max_pred=8, vocab_size=1000, split="test")
write_vocab(os.path.join(t, "v.txt"), 1000)
cfg = write_bert_config(os.path.join(t, "c.json"), vocab_size=1000, hidden_size=256, num_hidden_layers=2,
                        num_attention_heads=4, intermediate_size=1024)
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
for extra in os.environ["DP_CASES"].split(";"):
    cmds = [[sys.executable, "train.py", "--task", "bert", "--data", d, "--dict", os.path.join(t, "v.txt"),
             "--config_file", cfg, "--max-sentences", "8", "--valid-subset", "test", "--max-update", "4",
             "--distributed-backend", "gloo", "--save-dir", os.path.join(t, "ck"), "--no-save",
             "--distributed-init-method", "tcp://127.0.0.1:%d" % port, "--distributed-world-size", "2",
             "--distributed-rank", str(r), "--distributed-gpus", "1", "--device-id", "0", "--check-consistency", "1",
             "--fast-stat-sync", "--lr", "1e-3"] + extra.split() for r in range(2)]
    ps = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for c in cmds]
    outs = [p.communicate(timeout=300)[0] for p in ps]
    ok = all(p.returncode == 0 for p in ps)
    err = [l for l in outs[0].splitlines() if "diverged" in l or "Error" in l][-1:]
    print("CASE", repr(extra), "OK" if ok else "FAIL", err, flush=True)
    port += 1
