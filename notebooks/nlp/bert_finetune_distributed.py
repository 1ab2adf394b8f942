# Databricks notebook source
# MAGIC %md
# MAGIC ## BERT-base fine-tuning (seq 128) with a HorovodRunner-style launcher
# MAGIC
# MAGIC `HorovodRunner(np=8).run(main)` — inside `main` the Horovod-style facade
# MAGIC (`hvd.init / DistributedOptimizer / broadcast_parameters`) is backed by the RCCL reducer.

# COMMAND ----------

import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__) if "__file__" in dir() else ".", "../..")))

import torch

SMOKE = os.environ.get("DDL_NOTEBOOK_SMOKE") == "1"

# COMMAND ----------


def main(steps=20, batch=64, seq=128, smoke=False):
    import time
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.data import SyntheticTokens
    from databricks_distributed_deep_learning_amd.models import bert_base, cast_params
    from databricks_distributed_deep_learning_amd.models.bert import BertConfig, BertForSequenceClassification
    from databricks_distributed_deep_learning_amd.parallel import hvd
    hvd.init()
    dev = torch.device("cuda", hvd.local_rank()) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(0)
    if smoke:
        model = BertForSequenceClassification(BertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                                         intermediate_size=128, vocab_size=1000))
    else:
        model = bert_base(num_labels=2)
    model = model.to(dev)
    if dev.type == "cuda":
        cast_params(model, torch.bfloat16)
    opt = hvd.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=2e-5),
                                   named_parameters=model.named_parameters())
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    data = SyntheticTokens(batch, seq, 1000 if smoke else 30522, 2, dev, rank=hvd.rank())
    t0 = time.time()
    for step in range(steps):
        b = data.next()
        opt.zero_grad()
        loss, _ = model(b["input_ids"], b["attention_mask"], None, b["labels"])
        loss.backward()
        opt.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    return {"loss": float(loss), "samples_per_sec_per_rank": steps * batch / dt, "world": hvd.size()}

# COMMAND ----------


from databricks_distributed_deep_learning_amd.parallel import HorovodRunner

if __name__ == "__main__":
    if SMOKE or not torch.cuda.is_available():
        print(HorovodRunner(np=2, use_gpu=False).run(main, steps=2, batch=2, seq=16, smoke=True))
    else:
        print(HorovodRunner(np=torch.cuda.device_count()).run(main))
