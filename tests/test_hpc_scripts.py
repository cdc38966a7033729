"""Cluster orchestration scripts tested without a cluster: fake sbatch / srun /
scontrol / squeue / torchrun / mpiexec / amd-smi executables on PATH record their
argv, and the job scripts' generated command lines are asserted."""
import os
import stat
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HPC = ROOT / "hpc_files"

FAKES = {
    "sbatch": 'echo "sbatch $*" >> "$FAKE_LOG"',
    "squeue": "exit 0",
    "scontrol": 'if [ "$1 $2" = "show hostname" ]; then echo "$3" | tr "," "\\n"; fi',
    # srun: drop its own options, then run the command (so launcher scripts really execute)
    "srun": '''echo "srun $*" >> "$FAKE_LOG"
while [ $# -gt 0 ]; do case "$1" in -w|-N|-n|-o|--ntasks-per-node) shift 2;; --*|-*) shift;; *) break;; esac; done
exec "$@"''',
    "torchrun": 'echo "torchrun $*" >> "$FAKE_LOG"',
    "mpiexec": 'echo "mpiexec $*" >> "$FAKE_LOG"',
    "fakepython": 'echo "python $*" >> "$FAKE_LOG"',
    "amd-smi": 'if [ "$1" = list ]; then for i in 0 1 2 3; do echo "GPU: $i"; echo "  BDF: x"; done; fi',
}


@pytest.fixture
def fakeenv(tmp_path):
    b = tmp_path / "bin"
    b.mkdir()
    for name, body in FAKES.items():
        p = b / name
        p.write_text("#!/bin/bash\n" + body + "\n")
        p.chmod(p.stat().st_mode | stat.S_IEXEC)
    log = tmp_path / "calls.log"
    log.write_text("")
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    env = {k: v for k, v in os.environ.items() if not k.startswith(("SLURM", "ROCR", "HIP_VIS", "CUDA_VIS"))}
    env.update(PATH=f"{b}:{env['PATH']}", FAKE_LOG=str(log), SCRATCH=str(scratch), DTP_SKIP_VENV="1",
               USER="tester", HOME=str(tmp_path))
    return env, log, scratch


def run(cmd, env, cwd=HPC, ok=True, inp=None):
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=60, input=inp)
    if ok:
        assert r.returncode == 0, r.stdout + r.stderr
    return r


def _sbatch_line(out: str) -> str:
    return [l for l in out.splitlines() if l.startswith("sbatch ")][-1]


def test_distributed_torchrun_submission(fakeenv):
    env, log, scratch = fakeenv
    r = run(["bash", "job_submitter.sh", "-j", "distributed", "-W", "torchrun", "-g", "8", "-c", "4", "-N", "2",
             "-G", "mi355x", "-e", "exp1", "-p", "gpu", "--print-only"], env)
    line = _sbatch_line(r.stdout)
    for frag in ["--ntasks-per-node=1", "--cpus-per-task=32", "--gres=gpu:mi355x:8", "--nodes=2",
                 "--partition=gpu", "which_distributed=torchrun", "cmd=python demo.py --backend=nccl --torchrun",
                 "virtual_env_hpc_files/distributed_dispatcher.sh", "HSA_ENABLE_IPC_MODE_LEGACY=0"]:
        assert frag in line, (frag, line)
    assert (scratch / ROOT.name / "exp1" / "checkpoints").is_dir()


def test_lightning_and_mpi_submission(fakeenv):
    env, log, _ = fakeenv
    for w in ("lightning", "mpi"):
        r = run(["bash", "job_submitter.sh", "-j", "distributed", "-W", w, "-g", "4", "-n", "3", "--print-only",
                 "-C", str(HPC / ("lightning_configs.txt" if w == "lightning" else "mpi_configs.txt"))], env)
        line = _sbatch_line(r.stdout)
        assert "--ntasks-per-node=4" in line and "--nodes=3" in line and "--cpus-per-task=2" in line


def test_standard_and_sweep_submission(fakeenv):
    env, log, _ = fakeenv
    line = _sbatch_line(run(["bash", "job_submitter.sh", "-g", "1", "-N", "4", "--print-only"], env).stdout)
    assert "--nodes=1" in line and "standard_job.sh" in line and "--gres=gpu:1" in line
    env2 = dict(env, DTP_SWEEP_ID="abc123", DTP_N_SWEEPS="5")
    line = _sbatch_line(run(["bash", "job_submitter.sh", "-j", "sweep", "-C", str(HPC / "sweep_cmd.txt"),
                             "--print-only"], env2).stdout)
    assert "--array 1-5%10" in line and "cmd=wandb agent --count 1 WANDB_USERNAME/PROJECT_ROOT/abc123" in line


def test_real_submit_and_data_tarball(fakeenv):
    env, log, scratch = fakeenv
    proj = scratch / ROOT.name
    (proj / "datasets").mkdir(parents=True)
    (proj / "datasets" / "a.txt").write_text("x")
    run(["bash", "job_submitter.sh", "-j", "distributed", "-W", "torchrun", "-g", "2", "-d", "datasets", "-y"], env)
    calls = log.read_text()
    assert "sbatch " in calls and "distributed_dispatcher.sh" in calls
    tar = proj / "tar_ball_datasets.tar"
    assert tar.exists() and calls.strip().endswith(str(tar))


@pytest.mark.parametrize("args,msg", [
    (["-g", "0"], "gpus must be"), (["-j", "nope"], "supported job types"),
    (["-j", "distributed"], "which-distributed"), (["-G", "v100l"], "supported gpu types"),
    (["-m", "10T"], "memory"), (["--bogus"], "unknown argument")])
def test_validation(fakeenv, args, msg):
    env, _, _ = fakeenv
    r = run(["bash", "job_submitter.sh", *args, "--print-only"], env, ok=False)
    assert r.returncode != 0 and msg in r.stderr


def test_requires_scratch(fakeenv):
    env, _, _ = fakeenv
    env = {k: v for k, v in env.items() if k != "SCRATCH"}
    r = run(["bash", "job_submitter.sh", "--print-only"], env, ok=False)
    assert "SCRATCH" in r.stderr


def _job_env(env, scratch, which, cmd, nodes="n1,n2"):
    return dict(env, source_dir=str(ROOT), scratch_dir=str(scratch), which_distributed=which, cmd=cmd,
                SLURM_NODELIST=nodes, SLURM_JOB_NUM_NODES=str(len(nodes.split(","))), SLURM_JOB_ID="77",
                MASTER_ADDR="n1", PYTHON=str(Path(env["PATH"].split(":")[0]) / "fakepython"))


def test_dispatcher_torchrun_per_node(fakeenv):
    env, log, scratch = fakeenv
    e = _job_env(env, scratch, "torchrun", "python demo.py --backend=nccl --torchrun")
    run(["bash", str(HPC / "virtual_env_hpc_files" / "distributed_dispatcher.sh"), ""], e)
    tr = [l for l in log.read_text().splitlines() if l.startswith("torchrun")]
    assert len(tr) == 2  # one launcher per node
    for l in tr:
        assert "--nproc_per_node 4 --nnodes 2" in l  # 4 GPUs from the fake amd-smi
        assert "--rdzv_backend=c10d --rdzv_endpoint=n1:2345 --max_restarts=3" in l
        assert l.endswith("demo.py --backend=nccl --torchrun")


def test_torchrun_launcher_single_node_and_gpu_env(fakeenv):
    env, log, scratch = fakeenv
    e = _job_env(env, scratch, "torchrun", "python demo.py --torchrun", nodes="n1")
    e["ROCR_VISIBLE_DEVICES"] = "0,1,2,3,4,5,6,7"
    run(["bash", str(HPC / "virtual_env_hpc_files" / "distributed_dispatcher.sh"), ""], e)
    l = [l for l in log.read_text().splitlines() if l.startswith("torchrun")][0]
    assert "--nproc_per_node 8 --nnodes 1 --master_addr 127.0.0.1" in l


def test_launcher_rejects_non_python(fakeenv):
    env, log, scratch = fakeenv
    e = _job_env(env, scratch, "torchrun", "bash evil.sh", nodes="n1")
    r = run(["bash", str(HPC / "virtual_env_hpc_files" / "distributed_scripts" / "torchrun_launcher.sh"),
             "0", "8", "n1", "2345", ""], e, ok=False)
    assert "Command must be a python execution" in r.stderr


def test_lightning_launcher_rewrites_counts(fakeenv):
    env, log, scratch = fakeenv
    e = _job_env(env, scratch, "lightning", "python demo_pytorch_lightning.py --gpus 2 --steps 10 --nnodes=7")
    run(["bash", str(HPC / "virtual_env_hpc_files" / "distributed_scripts" / "lightning_launcher.sh"),
         "2", "8", ""], e)
    l = [l for l in log.read_text().splitlines() if l.startswith("python")][0]
    assert l == "python demo_pytorch_lightning.py --steps 10 --nnodes=2 --gpus=8"


def test_mpi_launcher(fakeenv):
    env, log, scratch = fakeenv
    e = _job_env(env, scratch, "mpi", "python demo_assume_started_with_mpiexec.py --backend=nccl")
    run(["bash", str(HPC / "virtual_env_hpc_files" / "distributed_dispatcher.sh"), ""], e)
    l = [l for l in log.read_text().splitlines() if l.startswith("mpiexec")][0]
    assert l.startswith("mpiexec -n 8 ") and "demo_assume_started_with_mpiexec.py --backend=nccl" in l


def test_standard_job_runs_command(fakeenv, tmp_path):
    env, log, scratch = fakeenv
    e = dict(env, source_dir=str(ROOT), scratch_dir=str(scratch), cmd=f"{tmp_path}/bin/fakepython demo.py --iters 3")
    run(["bash", str(HPC / "virtual_env_hpc_files" / "standard_job.sh"), ""], e)
    assert "python demo.py --iters 3" in log.read_text()


def test_count_sweeps_and_help(fakeenv):
    env, _, _ = fakeenv
    assert run(["bash", "count_sweeps.bash", "sweeper.yml"], env).stdout.strip() == "8"
    assert run(["bash", "count_sweeps.bash", "nope.yml"], env, ok=False).returncode != 0
    assert "Usage" in run(["bash", "job_submitter.sh", "-h"], env).stdout


def test_scripts_are_valid_bash():
    for p in list(HPC.rglob("*.sh")) + list((ROOT / "interactive_job_cmds").glob("*.sh")) + [HPC / "count_sweeps.bash"]:
        r = subprocess.run(["bash", "-n", str(p)], capture_output=True, text=True)
        assert r.returncode == 0, (p, r.stderr)


def test_singularity_job_builds_the_container_command(fakeenv, tmp_path):
    """The Singularity/Apptainer job: the container is staged to the node's
    temp dir and run with --rocm (not --nv), the results / data / tmp / source bind
    mounts, the experiment command, and the RCCL/IPC environment passed inside."""
    env, log, scratch = fakeenv
    fake = tmp_path / "bin" / "apptainer"
    fake.write_text('#!/bin/bash\necho "apptainer $* | ipc=$SINGULARITYENV_HSA_ENABLE_IPC_MODE_LEGACY '
                    'procid=$SINGULARITYENV_SLURM_PROCID" >> "$FAKE_LOG"\n')
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    rs = tmp_path / "bin" / "rsync"  # rsync may be missing on the test host: copy the last two args
    rs.write_text('#!/bin/bash\ncp "${@: -2:1}" "${@: -1}"\n')
    rs.chmod(rs.stat().st_mode | stat.S_IEXEC)
    image = tmp_path / "dtp_rocm.sif"
    image.write_text("image")
    node_tmp = tmp_path / "node"
    e = dict(env, source_dir=str(ROOT), scratch_dir=str(scratch), exp_name="exp1", singularity_container=str(image),
             SLURM_TMPDIR=str(node_tmp), SLURM_JOB_ID="42", SLURM_PROCID="3",
             cmd="python demo.py --iters 3 --backend=nccl")
    run(["bash", str(HPC / "singularity_hpc_files" / "standard_job.sh"), "", "code"], e)
    line = [l for l in log.read_text().splitlines() if l.startswith("apptainer ")][-1]
    assert line.startswith("apptainer run --rocm ") and "--nv" not in line
    assert f"-B {scratch}/exp1:/results" in line and f"-B {node_tmp}/data:/data" in line
    assert f"-B {ROOT}:/code --pwd /code" in line
    assert f"{node_tmp}/dtp_rocm.sif python demo.py --iters 3 --backend=nccl" in line
    assert line.endswith("ipc=0 procid=3")
    assert (node_tmp / "dtp_rocm.sif").exists() and (scratch / "exp1").is_dir()
