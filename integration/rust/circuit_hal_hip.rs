// The circuit side of the HIP backend: one file per circuit crate, behind `feature = "hip"`.
//   risc0/circuit/rv32im/src/prove/hal/hip.rs     (counterpart of prove/hal/cuda.rs)
//   risc0/circuit/recursion/src/prove/hal/hip.rs  (counterpart of prove/hal/cuda.rs)
// Both are shown here; split them at the marked line.
//
// eval_check runs on the device (r0hip_eval_check: the constraint program generated for
// gfx950 from the circuit, tools/gen_eval_check.py), and so do both circuits' accumulations:
// rv32im's three phases (r0hip_rv32im_accum: stepAccum generated from the reference's
// step_TopAccum, the scan and finalizeAccum) and the recursion circuit's
// (r0hip_recursion_accum), and both circuits' witness generation: rv32im's stepExec
// (r0hip_rv32im_witgen: step_Top generated from the reference's steps.cpp, two phases split
// at tableSplitCycle, the same RawExecBuffers / RawPreflightTrace the CUDA HAL passes) and the
// recursion circuit's (r0hip_recursion_witgen).
//
// Selection (one arm each):
//   circuit/rv32im/src/prove/mod.rs:45-55       if #[cfg(feature = "hip")] { self::hal::hip::segment_prover() }
//   circuit/recursion/src/prove/mod.rs:82-93    if #[cfg(feature = "hip")] { self::hal::hip::recursion_prover(hashfn) }
//
// NOT COMPILED IN THIS REPOSITORY (no Rust toolchain in the image).

// ======================= risc0/circuit/rv32im/src/prove/hal/hip.rs =======================
use std::{ffi::CString, rc::Rc};

use anyhow::Result;
use risc0_circuit_rv32im_sys::{RawBuffer, RawExecBuffers, RawPreflightTrace};
use risc0_core::{field::ExtElem as _, scope};
use risc0_sys::{
    ffi_wrap,
    hip::{r0hip_eval_check, r0hip_rv32im_accum, r0hip_rv32im_witgen},
};
use risc0_zkp::hal::{
    AccumPreflight, Buffer, CircuitHal,
    hip::{BufferImpl as HipBuffer, HipHal, HipHash, HipHashPoseidon2},
};

use super::{
    CircuitAccumulator, CircuitWitnessGenerator, MetaBuffer, PreflightTrace, SegmentProverImpl, StepMode,
};
use crate::{
    prove::{GLOBAL_MIX, GLOBAL_OUT, SegmentProver},
    zirgen::circuit::{ExtVal, REGISTER_GROUP_ACCUM, REGISTER_GROUP_CODE, REGISTER_GROUP_DATA, Val},
};

pub struct HipCircuitHal<HS: HipHash> {
    _hal: Rc<HipHal<HS>>, // keeps the device bound while the circuit HAL lives
}

impl<HS: HipHash> HipCircuitHal<HS> {
    pub fn new(_hal: Rc<HipHal<HS>>) -> Self {
        Self { _hal }
    }
}

fn raw_device<HS: HipHash>(m: &MetaBuffer<HipHal<HS>>) -> RawBuffer {
    RawBuffer { buf: m.buf.dev() as *const Val, rows: m.rows, cols: m.cols, checked: m.checked }
}

fn raw_preflight(p: &PreflightTrace) -> RawPreflightTrace {
    RawPreflightTrace {
        cycles: p.cycles.as_ptr(),
        txns: p.txns.as_ptr(),
        bigint_bytes: p.bigint_bytes.as_ptr(),
        txns_len: p.txns.len() as u32,
        bigint_bytes_len: p.bigint_bytes.len() as u32,
        table_split_cycle: p.table_split_cycle,
    }
}

impl<HS: HipHash> CircuitWitnessGenerator<HipHal<HS>> for HipCircuitHal<HS> {
    fn generate_witness(
        &self,
        mode: StepMode,
        preflight: &PreflightTrace,
        global: &MetaBuffer<HipHal<HS>>,
        data: &MetaBuffer<HipHal<HS>>,
    ) -> Result<()> {
        scope!("witgen");
        // prove/hal/cuda.rs:60-101 with the HIP kernels: device buffers, host preflight arrays
        let cycles = preflight.cycles.len();
        assert_eq!(cycles, data.rows);
        let buffers = RawExecBuffers { global: raw_device(global), data: raw_device(data) };
        let pf = raw_preflight(preflight);
        ffi_wrap(|| unsafe {
            r0hip_rv32im_witgen(mode as u32, &buffers as *const _ as *const _, &pf as *const _ as *const _, cycles as u32)
        })
    }
}

impl<HS: HipHash> CircuitAccumulator<HipHal<HS>> for HipCircuitHal<HS> {
    fn step_accum(
        &self,
        preflight: &PreflightTrace,
        data: &MetaBuffer<HipHal<HS>>,
        accum: &MetaBuffer<HipHal<HS>>,
        global: &MetaBuffer<HipHal<HS>>,
        mix: &MetaBuffer<HipHal<HS>>,
    ) -> Result<()> {
        scope!("accumulate");
        let cycles = preflight.cycles.len();
        // all three phases of risc0_circuit_rv32im_cuda_accum (ffi.cu:362-514) on the device:
        // the per-cycle stepAccum generated from the reference's step_TopAccum, the scan and
        // finalizeAccum. `accum` arrives INVALID-filled as the CUDA HAL allocates it, except
        // accum columns 0..11 of every BigInt cycle: WitnessGenerator::accum has already
        // scattered the BigIntAccumState there (witgen/mod.rs:182-205), and the step reads the
        // previous cycle's state from them at back 1. The step reads no other preflight data.
        assert_eq!(accum.rows, data.rows);
        ffi_wrap(|| unsafe {
            r0hip_rv32im_accum(
                data.buf.dev(),
                accum.buf.dev(),
                global.buf.dev(),
                mix.buf.dev(),
                accum.rows,
                accum.cols,
                cycles,
            )
        })
    }
}

impl<HS: HipHash> CircuitHal<HipHal<HS>> for HipCircuitHal<HS> {
    fn accumulate(
        &self,
        _preflight: &AccumPreflight,
        _ctrl: &HipBuffer<Val>,
        _io: &HipBuffer<Val>,
        _data: &HipBuffer<Val>,
        _mix: &HipBuffer<Val>,
        _accum: &HipBuffer<Val>,
        _steps: usize,
    ) {
        // rv32im accumulates through CircuitAccumulator::step_accum (as the CUDA HAL does)
    }

    fn eval_check(
        &self,
        check: &HipBuffer<Val>,
        groups: &[&HipBuffer<Val>],
        globals: &[&HipBuffer<Val>],
        poly_mix: ExtVal,
        po2: usize,
        steps: usize,
    ) {
        scope!("eval_check");
        assert_eq!(steps, 1 << po2);
        // r0hip takes the groups in tap-group order (accum 0, code 1, data 2) and expands the
        // poly_mix powers itself (zirgen/info.rs POLY_MIX_POWERS are compiled in)
        let g = [
            groups[REGISTER_GROUP_ACCUM].dev() as *const u32,
            groups[REGISTER_GROUP_CODE].dev() as *const u32,
            groups[REGISTER_GROUP_DATA].dev() as *const u32,
        ];
        let pm = poly_mix.to_u32_words();
        let name = CString::new("rv32im").unwrap();
        ffi_wrap(|| unsafe {
            r0hip_eval_check(
                name.as_ptr(),
                check.dev(),
                g.as_ptr(),
                globals[GLOBAL_MIX].dev(),
                globals[GLOBAL_OUT].dev(),
                pm.as_ptr(),
                po2 as u32,
            )
        })
        .unwrap();
    }
}

pub type HipCircuitHalPoseidon2 = HipCircuitHal<HipHashPoseidon2>;

pub fn segment_prover() -> Result<Box<dyn SegmentProver>> {
    let hal_factory = || {
        let hal = Rc::new(HipHal::<HipHashPoseidon2>::new());
        let circuit_hal = Rc::new(HipCircuitHalPoseidon2::new(hal.clone()));
        (hal, circuit_hal)
    };
    Ok(Box::new(SegmentProverImpl::new(hal_factory)))
}

#[cfg(test)]
mod tests {
    // eval_check on the device against the CPU circuit HAL on the same random buffers, as
    // prove/hal/cuda.rs tests do with EvalCheckParams (po2 = 4 .. 10, every cycle).
    use std::rc::Rc;

    use risc0_core::field::baby_bear::BabyBear;
    use risc0_zkp::{
        core::hash::sha::Sha256HashSuite,
        hal::{Hal, cpu::CpuHal, hip::HipHalSha256},
    };

    use super::*;
    use crate::prove::hal::{cpu::CpuCircuitHal, cuda::tests::EvalCheckParams};

    #[test]
    fn eval_check_matches_cpu() {
        for po2 in [4, 8, 10] {
            let p = EvalCheckParams::new(po2);
            let cpu_hal: CpuHal<BabyBear> = CpuHal::new(Sha256HashSuite::new_suite());
            let gpu_hal = Rc::new(HipHalSha256::new());
            let check_cpu = {
                let check = cpu_hal.alloc_elem("check", 4 * p.domain);
                let bufs = [&p.accum, &p.code, &p.data].map(|v| cpu_hal.copy_from_elem("g", v));
                let (mix, out) = (cpu_hal.copy_from_elem("mix", &p.mix), cpu_hal.copy_from_elem("out", &p.out));
                CpuCircuitHal.eval_check(&check, &[&bufs[0], &bufs[1], &bufs[2]], &[&mix, &out], p.poly_mix, po2, p.steps);
                check.to_vec()
            };
            let check_gpu = {
                let check = gpu_hal.alloc_elem("check", 4 * p.domain);
                let bufs = [&p.accum, &p.code, &p.data].map(|v| gpu_hal.copy_from_elem("g", v));
                let (mix, out) = (gpu_hal.copy_from_elem("mix", &p.mix), gpu_hal.copy_from_elem("out", &p.out));
                HipCircuitHal::new(gpu_hal.clone())
                    .eval_check(&check, &[&bufs[0], &bufs[1], &bufs[2]], &[&mix, &out], p.poly_mix, po2, p.steps);
                check.to_vec()
            };
            assert_eq!(check_cpu, check_gpu, "po2 = {po2}");
        }
    }
}

// The recursion circuit's HAL is integration/rust/recursion_circuit_hal_hip.rs.
