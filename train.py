"""Box-side pretraining driver with the command line of the reference's ``train_concap_struc.py``
(argparse surface :68-138, setup :140-448, training loop :466-589, evaluation :612-688, per-epoch
checkpoints :691-705), running the MI355X step: ``k3m_amd.trainer.Trainer`` (the HIP engine, fused AdamW
launches, RCCL all-reduce overlapped with backward through ``k3m_amd.ddp.GradAllReducer``).

    python train.py --data_dir DIR --output_dir OUT --file_name NAME [reference options]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ... (one rank per GPU)

Same files as the reference: ``<output_dir>/<config_file>`` (BertConfig JSON), ``<output_dir>/
<pretrained_model_weights>`` (the BERT weight-name list for the x0.1 lr groups and ``--freeze``),
``<output_dir>/k3m_<model_name>_<layers>l_<heads>h/`` receiving ``hyperparamter.txt`` and the per-epoch
``K3M_struc_presample-<p>_epoch-<e>.bin/.tar`` in the reference layout (k3m_amd/checkpoint.py).  Log lines
follow the reference's format.

Differences, each stated:
* the step is the fused HIP engine, not nn.Module autograd; ``--fp16`` / ``--apex_fast`` select the bf16
  encoder with fp32 master weights and apex FusedAdam semantics (k3m_amd/trainer.py) instead of apex amp;
* records come from a ``k3m_amd.loaders.write_records`` directory or a raw product TSV (the tensorpack
  LMDB container is not read);
* build-side options, all prefixed ``--k3m_``: ``--k3m_char_tokenizer`` (no vocab.txt offline),
  ``--k3m_synthetic_regions SEED`` (region features for TSV rows), ``--k3m_no_shuffle``,
  ``--k3m_max_steps N``, ``--k3m_loss_log PATH`` (one JSON line per step), and the parity harness
  ``--k3m_parity_case NPZ``: every step feeds the fixture's recorded batch with its gumbel noise and LPM
  negatives, dropout off (the golden vectors were recorded with model.eval(); tests/test_gpu_train_driver.py).
"""
import argparse
import json
import logging
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

logging.basicConfig(format="%(asctime)s %(levelname)-4s [%(filename)s:%(lineno)s]  %(message)s",
                    datefmt="%Y/%m/%d %H:%M:%S", level=logging.INFO)
logger = logging.getLogger(__name__)


def get_parser(argv=None):
    """The reference's options (train_concap_struc.py:68-138), same names, types and defaults."""
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", required=True, type=str, help="directory of the training records")
    p.add_argument("--output_dir", required=True, type=str, help="config / weight-name files; checkpoints go below")
    p.add_argument("--file_name", required=True, type=str, help="record file name ('{}' -> train+valid / valid)")
    p.add_argument("--model_name", default="bert-base-uncased", type=str)
    p.add_argument("--pretrained_model_path", default=None, type=str,
                   help="directory with vocab.txt and pytorch_model.bin (BERT init, lr x0.1 groups)")
    p.add_argument("--config_file", default="bert_base_6layer_6conect.json", type=str)
    p.add_argument("--pretrained_model_weights", default="bert-base-uncased_weight_name.json", type=str)
    p.add_argument("--file_checkpoint", default="", type=str, help="resume from a .tar")
    p.add_argument("--file_state_dict", default="", type=str, help="load model weights from a .bin")
    p.add_argument("--log_steps", default=1, type=int)
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--cache", default=5000, type=int)
    p.add_argument("--do_train", action="store_true")
    p.add_argument("--do_eval", action="store_true")
    p.add_argument("--seed", default=42, type=int)
    p.add_argument("--on_memory", action="store_true")
    p.add_argument("--local_rank", default=-1, type=int)
    p.add_argument("--train_batch_size", default=8, type=int)
    p.add_argument("--eval_batch_size", default=8, type=int)
    p.add_argument("--learning_rate", default=1e-4, type=float)
    p.add_argument("--num_train_epochs", default=6.0, type=float)
    p.add_argument("--start_epoch", default=0, type=float)
    p.add_argument("--no_cuda", action="store_true")
    p.add_argument("--num_workers", default=2, type=int)
    p.add_argument("--if_pre_sampling", default=1, type=int)
    p.add_argument("--with_coattention", action="store_true")
    p.add_argument("--objective", default=2, type=int)
    p.add_argument("--freeze", default=-1, type=int)
    p.add_argument("--warmup_proportion", default=0.1, type=float)
    p.add_argument("--gradient_accumulation_steps", default=1, type=int)
    p.add_argument("--adam_epsilon", default=1e-8, type=float)
    p.add_argument("--loss_img_weight", default=1, type=float)
    p.add_argument("--fp16", action="store_true")
    p.add_argument("--apex_fast", action="store_true")
    p.add_argument("--loss_scale", default=0, type=float)
    p.add_argument("--do_lower_case", default=True, type=bool)
    p.add_argument("--max_seq_length", default=36, type=int)
    p.add_argument("--max_seq_length_pv", default=128, type=int)
    p.add_argument("--max_num_pv", default=20, type=int)
    p.add_argument("--max_region_length", default=36, type=int)
    p.add_argument("--dynamic_attention", action="store_true")
    p.add_argument("--visual_target", default=0, type=int)
    p.add_argument("--num_negative", default=255, type=int)
    # build-side options (module docstring)
    p.add_argument("--k3m_char_tokenizer", action="store_true")
    p.add_argument("--k3m_synthetic_regions", default=None, type=int)
    p.add_argument("--k3m_no_shuffle", action="store_true")
    p.add_argument("--k3m_max_steps", default=0, type=int)
    p.add_argument("--k3m_loss_log", default="", type=str)
    p.add_argument("--k3m_parity_case", default="", type=str)
    return p.parse_args(argv)


def _trunc(x):
    # the reference logs int(value * 1000) / 1000 (:542-553)
    return int(float(x) * 1000) / 1000


def _parity_inputs(path, dev):
    """Recorded batch, gumbel noise and LPM negative tables of a golden case (tests/golden/make_golden.py)."""
    d = np.load(path, allow_pickle=False)
    batch = {k[3:]: torch.from_numpy(d[k]).to(dev) for k in d.files if k.startswith("in/")}
    B, T = batch["input_ids"].shape
    P, R = batch["input_ids_pv"].shape[1], batch["image_feat"].shape[1]
    rng = np.random.default_rng(int(d["noise_seed"]))
    noise = {k: torch.from_numpy((-np.log(rng.standard_exponential(s))).astype(np.float32)).to(dev)
             for k, s in [("v", (B, R, 3, 1024)), ("t", (B, T, 3, 768)), ("pv", (B, P, 3, 768))]}
    return batch, noise, torch.from_numpy(d["ent_neg"]).to(dev), torch.from_numpy(d["val_neg"]).to(dev), \
        int(d["mode"])


def main(argv=None):
    args = get_parser(argv)
    from k3m_amd.config import BertConfig
    from k3m_amd.trainer import Trainer, bert_lr_mult
    from k3m_amd import checkpoint as C

    if args.no_cuda:
        raise SystemExit("train.py runs the HIP engine; --no_cuda has no CPU path in this build")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.local_rank == -1 and world > 1:
        args.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.local_rank == -1:
        dev = torch.device("cuda")
        n_gpu = torch.cuda.device_count()
    else:
        torch.cuda.set_device(args.local_rank)
        dev = torch.device("cuda", args.local_rank)
        n_gpu = 1
        torch.distributed.init_process_group(backend="nccl", device_id=dev)
    distributed = args.local_rank != -1
    logger.info(f"device: {dev} n_gpu: {n_gpu}, distributed training: {distributed}, 16-bits training: {args.fp16}")

    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    torch.cuda.manual_seed_all(args.seed)
    default_gpu = (not distributed) or torch.distributed.get_rank() == 0

    config = BertConfig.from_json_file(os.path.join(args.output_dir, args.config_file))
    model_path = f"k3m_{args.model_name}_{config.num_hidden_layers}l_{config.num_attention_heads}h"
    output_model_path = os.path.join(args.output_dir, model_path)
    if default_gpu:
        os.makedirs(output_model_path, exist_ok=True)
        with open(os.path.join(output_model_path, "hyperparamter.txt"), "w") as f:
            print(args, file=f)
            print("\n", file=f)
            print(config, file=f)
    config.v_target_size = 1601 if args.visual_target == 0 else 2048
    config.visual_target = args.visual_target
    if "roberta" in args.model_name:
        config.model = "roberta"
    if args.freeze > config.t_biattention_id[0]:
        # the reference then sets config.fixed_t_layer = t_biattention_id[0] (:206-207): the text layers below the
        # first co-attention run under no_grad, which also cuts the embeddings' gradient.  The wide engine does not
        # implement that truncated backward; refuse instead of training a different model.
        raise SystemExit("--freeze %d > t_biattention_id[0] = %d (fixed_t_layer) is not supported by the MI355X "
                         "engine; use --freeze <= %d" % (args.freeze, config.t_biattention_id[0],
                                                         config.t_biattention_id[0]))
    config.with_coattention = args.with_coattention
    config.dynamic_attention = args.dynamic_attention
    config.if_pre_sampling = args.if_pre_sampling
    config.num_negative = args.num_negative

    parity = None
    if args.k3m_parity_case:
        parity = _parity_inputs(args.k3m_parity_case, dev)
        config.if_pre_sampling = parity[4]

    train_batch_size = args.train_batch_size // args.gradient_accumulation_steps
    if distributed:
        train_batch_size //= torch.distributed.get_world_size()

    tokenizer = None
    if parity is None:
        if args.k3m_char_tokenizer:
            from k3m_amd.loaders import CharTokenizer
            tokenizer = CharTokenizer()
        else:
            from pytorch_transformers.tokenization_bert import BertTokenizer
            tokenizer = BertTokenizer.from_pretrained(args.pretrained_model_path, do_lower_case=args.do_lower_case)
            tokenizer.do_basic_tokenize = False

    # parameter groups (:352-389) and --freeze (:243-260)
    from k3m_amd.params import param_spec
    names = [n for n, _ in param_spec(config)]
    wpath = os.path.join(args.output_dir, args.pretrained_model_weights)
    bert_weight_name = json.load(open(wpath, "r", encoding="utf-8")) if os.path.exists(wpath) else []
    frozen = []
    if args.freeze != -1:
        keep = [n for n in bert_weight_name if "embeddings" in n or
                ("encoder" in n and int(n.split(".")[2]) <= args.freeze)]
        # the reference's freeze loop runs on the unwrapped model, before the DDP wrap (:254-257 vs :308):
        # the key never carries "module." there, in any mode
        frozen = [n for n in names if n[12:] in set(keep)]
    lr_mult = bert_lr_mult(names, bert_weight_name, ddp=distributed) if args.pretrained_model_path else None

    num_dataset = 0
    train_loader = valid_loader = None
    if args.do_train and parity is None:
        from vilbert_k3m.datasets import ConceptCapLoaderTrain_struc, ConceptCapLoaderVal_struc
        import tensorpack.dataflow as td
        kw = dict(max_seq_len=args.max_seq_length, max_seq_len_pv=args.max_seq_length_pv, max_num_pv=args.max_num_pv,
                  max_region_len=args.max_region_length, visual_target=args.visual_target,
                  v_target_size=config.v_target_size, objective=args.objective, serializer=td.LMDBSerializer,
                  device=dev, synthetic_regions=args.k3m_synthetic_regions, seed=args.seed)
        train_loader = ConceptCapLoaderTrain_struc(args.data_dir, args.file_name.format("train+valid"), tokenizer,
                                                   batch_size=train_batch_size, num_workers=args.num_workers,
                                                   local_rank=args.local_rank, cache=args.cache, **kw)
        if args.k3m_no_shuffle:
            train_loader.shuffle = False
        num_dataset = train_loader.num_dataset
        if args.do_eval:
            valid_loader = ConceptCapLoaderVal_struc(args.data_dir, args.file_name.format("valid"), tokenizer,
                                                     batch_size=args.eval_batch_size, **kw)
    elif parity is not None:
        num_dataset = int(parity[0]["input_ids"].shape[0]) * max(1, args.k3m_max_steps)

    num_train_optimization_steps = int(num_dataset / args.train_batch_size / args.gradient_accumulation_steps) * \
        int(args.num_train_epochs - args.start_epoch)
    mixed = args.fp16 or args.apex_fast
    trainer = Trainer(config, dev, lr=args.learning_rate, warmup_steps=args.warmup_proportion * num_train_optimization_steps,
                      total_steps=num_train_optimization_steps, seed=args.seed, init=True,
                      dtype="bf16" if mixed else "fp32", optimizer="fused_adam" if mixed else "adamw",
                      lr_schedule="warmup_linear_fp16" if args.fp16 else "warmup_linear",
                      warmup_proportion=args.warmup_proportion, accum_steps=args.gradient_accumulation_steps,
                      lr_mult=lr_mult, frozen_names=frozen, objective=args.objective, eps=args.adam_epsilon,
                      loss_img_weight=args.loss_img_weight)
    fp = trainer.engine.fp
    if args.pretrained_model_path:
        sd = torch.load(os.path.join(args.pretrained_model_path, "pytorch_model.bin"), map_location="cpu",
                        weights_only=True)
        sd = {(k.replace("gamma", "weight").replace("beta", "bias"))[5 if k.startswith("bert.") else 0:]: v
              for k, v in sd.items()}
        C.load_model_state_dict(fp, sd, strict=False)
    if args.file_state_dict:
        C.load_model_state_dict(fp, torch.load(args.file_state_dict, map_location="cpu", weights_only=True),
                                strict=False)
        logger.info("Successfully loaded model state dict ...")
    if args.file_checkpoint and os.path.exists(args.file_checkpoint):
        trainer.load_checkpoint(args.file_checkpoint)
        logger.info("Successfully loaded model checkpoint ...")
    if distributed:
        from k3m_amd.ddp import GradAllReducer
        trainer.ddp = GradAllReducer(fp, comm_dtype=torch.bfloat16 if mixed else None)
        trainer.ddp.broadcast_params(fp)
    if parity is not None:
        trainer.dropout = False

    if default_gpu:
        logger.info("***** Running training *****")
        logger.info("  Num examples = %d", num_dataset)
        logger.info("  Batch size = %d", args.train_batch_size)
        logger.info("  Num steps = %d", num_train_optimization_steps)

    loss_log = open(args.k3m_loss_log, "w") if (args.k3m_loss_log and default_gpu) else None
    steps_done = 0
    for epoch in range(int(args.start_epoch), int(args.num_train_epochs)):
        if not args.do_train:
            break
        if parity is not None:
            it = ((parity[0], None) for _ in range(max(1, args.k3m_max_steps)))
        else:
            it = train_loader.batches()
        for step, (batch, _ids) in enumerate(it):
            if parity is not None:
                out = trainer.step(batch, noise=parity[1], ent_neg=parity[2], val_neg=parity[3])
            else:
                out = trainer.step(batch)
            vals = {k: float(out[k]) for k in ("loss", "masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv",
                                               "loss_lpm", "next_sentence_loss")}
            vals["masked_img_loss"] *= args.loss_img_weight
            if (step + 1) % args.log_steps == 0 and default_gpu:
                logger.info(f"[Epoch-{epoch} Step-{step}] loss: {_trunc(vals['loss'])} "
                            f"loss_t: {_trunc(vals['masked_lm_loss'])}, loss_v: {_trunc(vals['masked_img_loss'])}, "
                            f"loss_pv: {_trunc(vals['masked_lm_loss_pv'])}, loss_tri: {_trunc(vals['loss_lpm'])}")
            if loss_log:
                loss_log.write(json.dumps(dict(epoch=epoch, step=step, lr=trainer.current_lr(), **vals)) + "\n")
                loss_log.flush()
            steps_done += 1
            if args.k3m_max_steps and steps_done >= args.k3m_max_steps:
                break
        trainer.finish()   # the epoch's outstanding label-count / loss checks (synchronising)
        if args.do_eval and valid_loader is not None:
            logger.info(f"[Epoch-{epoch}] Starting evaluation ...")
            for step, (batch, _ids) in enumerate(valid_loader.batches()):
                out = trainer.evaluate(batch)
                logger.info(f"[Eval] [Epoch-{epoch}] loss: {_trunc(out['loss'])} "
                            f"loss_t: {_trunc(out['masked_lm_loss'])}, "
                            f"loss_v: {_trunc(float(out['masked_img_loss']) * args.loss_img_weight)}, "
                            f"loss_pv: {_trunc(out['masked_lm_loss_pv'])}, loss_tri: {_trunc(out['loss_lpm'])}")
        if default_gpu:
            logger.info(f"[Epoch-{epoch}] saving model")
            base = os.path.join(output_model_path, f"K3M_struc_presample-{args.if_pre_sampling}_epoch-{epoch}")
            trainer.save_checkpoint(tar_path=base + ".tar", bin_path=base + ".bin")
        if args.k3m_max_steps and steps_done >= args.k3m_max_steps:
            break
    trainer.finish()
    if loss_log:
        loss_log.close()
    if distributed:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
