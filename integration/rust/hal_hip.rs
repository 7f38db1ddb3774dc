// risc0/zkp/src/hal/hip.rs — the `Hal` trait (risc0/zkp/src/hal/mod.rs:55-258) on MI355X
// through libr0hip, behind `feature = "hip"` (add `#[cfg(feature = "hip")] pub mod hip;` to
// risc0/zkp/src/hal/mod.rs next to `cuda`).
//
// Counterpart of risc0/zkp/src/hal/cuda.rs:461-1049, written for the r0hip C ABI rather than
// translated from it:
//   * device memory comes from r0hip_alloc (a size-keyed pool inside libr0hip, so the
//     Prover's many short-lived buffers cost no hipMalloc once warm), not from `cust`;
//   * `view_mut` moves only the viewed slice across PCIe (cuda.rs:366-373 copies the whole
//     raw buffer both ways);
//   * every call is synchronous on return (include/r0hip.h), exactly what the Prover
//     assumes of `view`/`get_at` after a kernel;
//   * `has_unified_memory()` is false: Merkle openings go through `gather_sample`
//     (prove/merkle.rs:111-129); `get_at` on a Merkle node heap reads a page-locked host
//     mirror of the heap, copied beside the next calls once hash_fold has built the root
//     (r0hip_memcpy_d2h_start; a tree's ~50 x 17 node reads would otherwise be one synchronous
//     copy each);
//   * an allocation gets device memory at its first device use: `gather_sample` into a
//     buffer that has none yet gathers straight to the host (r0hip_gather_sample_host) and
//     `view` reads those words — MerkleTreeProver::prove's sample (merkle.rs:111-129) is only
//     viewed, so its 350 openings per proof cost one call each instead of alloc, gather, view
//     and free; a device use first uploads the gathered words;
//   * combos_prepare / combos_divide are overridden with the device versions, as cuda.rs:
//     986-1048 does (one batched call for every chunk instead of one per divisor).
//
// NOT COMPILED IN THIS REPOSITORY (no Rust toolchain in the image). The same call sequence,
// driven over the same C symbols from Python, produces the golden seals:
// tests/hal_prover.py + tests/test_gpu_parity.py::test_per_op_abi_prover_matches_golden_seal.

use std::{cell::{Cell, RefCell}, ffi::CStr, marker::PhantomData, os::raw::c_void, rc::Rc, sync::OnceLock};

use parking_lot::{ReentrantMutex, ReentrantMutexGuard};
use risc0_core::{
    field::{
        Elem, ExtElem, RootsOfUnity,
        baby_bear::{BabyBear, BabyBearElem, BabyBearExtElem},
    },
    scope,
};
use risc0_sys::{ffi_wrap, hip::*};

use super::{Buffer, Hal, tracker};
use crate::core::{
    digest::Digest,
    hash::{HashSuite, poseidon_254::Poseidon254HashSuite, poseidon2::Poseidon2HashSuite, sha::Sha256HashSuite},
    log2_ceil,
};

/// One HAL per process at a time, as with the CUDA HAL (cuda.rs:46-50): libr0hip binds the
/// process to one device at the first r0hip_init.
fn device_lock() -> &'static ReentrantMutex<()> {
    static LOCK: OnceLock<ReentrantMutex<()>> = OnceLock::new();
    LOCK.get_or_init(|| ReentrantMutex::new(()))
}

fn check(err: *const std::os::raw::c_char) {
    ffi_wrap(|| err).unwrap();
}

/// The device ordinal this process proves on. r0vm starts one worker process per GPU
/// (r0vm/src/actors/mod.rs:449-462) with HIP_VISIBLE_DEVICES=<i>, so it is 0 there;
/// R0HIP_DEVICE overrides it for hosts that share one process over several devices.
fn device_ordinal() -> i32 {
    std::env::var("R0HIP_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0)
}

// ---------------------------------------------------------------------------------------
// Buffers

/// A device allocation: bytes from r0hip_alloc, returned to libr0hip's pool on drop. The
/// MemoryTracker (hal/mod.rs:292-317) sees it like the CUDA HAL's RawBuffer.
struct DeviceAlloc {
    name: &'static str,
    /// device memory, allocated at the first device use (`device`)
    ptr: Cell<*mut c_void>,
    bytes: usize,
    /// words gather_sample put straight on the host while the allocation had no device memory
    /// (the whole allocation): view/get_at read them, `device` uploads them first
    gathered: RefCell<Option<Vec<u32>>>,
    /// Merkle node heaps: hash_fold's root layer starts a copy of the whole allocation into
    /// `mirror` (page-locked) beside the Prover's next calls (`pending`); get_at reads the mirror
    /// once that copy has landed and one element synchronously until then. The only Hal methods
    /// that write a Buffer<Digest> are hash_rows and hash_fold, plus view_mut; all three settle
    /// the copy and clear `mirror_ok`.
    mirror: Cell<*mut c_void>,
    mirror_ok: Cell<bool>,
    pending: Cell<*mut c_void>,
}

impl DeviceAlloc {
    fn new(name: &'static str, bytes: usize) -> Self {
        assert!(bytes > 0, "empty allocation: {name}");
        tracker().lock().unwrap().alloc(bytes);
        Self { name, ptr: Cell::new(std::ptr::null_mut()), bytes, gathered: RefCell::new(None),
               mirror: Cell::new(std::ptr::null_mut()), mirror_ok: Cell::new(false),
               pending: Cell::new(std::ptr::null_mut()) }
    }

    /// the device memory, allocated now if this is the first device use; words gathered to the
    /// host are uploaded first (a device op may read them, and any may write the buffer)
    fn device(&self) -> *mut c_void {
        if self.ptr.get().is_null() {
            let (name, bytes) = (self.name, self.bytes);
            let mut ptr = std::ptr::null_mut();
            ffi_wrap(|| unsafe { r0hip_alloc(&mut ptr, bytes) })
                .unwrap_or_else(|e| panic!("allocation failed on {name}: {bytes} bytes: {e}"));
            self.ptr.set(ptr);
        }
        if let Some(g) = self.gathered.borrow_mut().take() {
            check(unsafe { r0hip_memcpy_h2d(self.ptr.get(), g.as_ptr() as *const c_void, g.len() * 4) });
        }
        self.ptr.get()
    }

    /// wait out a mirror copy in flight (before the allocation is written or freed)
    fn settle(&self) {
        let c = self.pending.replace(std::ptr::null_mut());
        if !c.is_null() {
            let mut done = 0;
            check(unsafe { r0hip_copy_finish(c, 1, &mut done) });
        }
    }

    /// the device copy was written: the mirror is stale
    fn written(&self) {
        self.settle();
        self.mirror_ok.set(false);
    }

    /// hash_fold built the root: copy the heap to the host beside the next calls
    fn mirror_start(&self) {
        self.written();
        if self.mirror.get().is_null() {
            let mut h = std::ptr::null_mut();
            check(unsafe { r0hip_host_alloc(&mut h, self.bytes) });
            self.mirror.set(h);
        }
        let mut c = std::ptr::null_mut();
        check(unsafe { r0hip_memcpy_d2h_start(self.mirror.get(), self.device(), self.bytes, &mut c) });
        self.pending.set(c);
        self.mirror_ok.set(true);
    }

    /// the mirror if its copy has landed
    fn host(&self) -> Option<*const u8> {
        if !self.mirror_ok.get() {
            return None;
        }
        let c = self.pending.get();
        if !c.is_null() {
            let mut done = 0;
            check(unsafe { r0hip_copy_finish(c, 0, &mut done) });
            if done == 0 {
                return None;
            }
            self.pending.set(std::ptr::null_mut());
        }
        Some(self.mirror.get() as *const u8)
    }
}

impl Drop for DeviceAlloc {
    fn drop(&mut self) {
        self.settle();
        tracker().lock().unwrap().free(self.bytes);
        if !self.ptr.get().is_null() {
            unsafe { r0hip_free(self.ptr.get()) };
        }
        if !self.mirror.get().is_null() {
            unsafe { r0hip_host_free(self.mirror.get()) };
        }
    }
}

/// Hal buffer: a typed window [offset, offset + size) onto a shared allocation.
#[derive(Clone)]
pub struct BufferImpl<T> {
    alloc: Rc<RefCell<DeviceAlloc>>,
    offset: usize,
    size: usize,
    _t: PhantomData<T>,
}

impl<T> BufferImpl<T> {
    fn new(name: &'static str, size: usize) -> Self {
        Self {
            alloc: Rc::new(RefCell::new(DeviceAlloc::new(name, size * std::mem::size_of::<T>()))),
            offset: 0,
            size,
            _t: PhantomData,
        }
    }

    fn from_slice(name: &'static str, slice: &[T]) -> Self {
        let buf = Self::new(name, slice.len());
        check(unsafe { r0hip_memcpy_h2d(buf.dev_void(), slice.as_ptr() as *const c_void, std::mem::size_of_val(slice)) });
        buf
    }

    fn dev_void(&self) -> *mut c_void {
        let base = self.alloc.borrow().device() as *mut u8;
        unsafe { base.add(self.offset * std::mem::size_of::<T>()) as *mut c_void }
    }

    /// Device address of element 0 of this window, as raw u32 words.
    pub fn dev(&self) -> *mut u32 {
        self.dev_void() as *mut u32
    }

    /// Device address of element `idx` of this window (cuda.rs:316-320 `as_device_ptr_with_offset`).
    pub fn dev_at(&self, idx: usize) -> *mut u32 {
        unsafe { (self.dev_void() as *mut u8).add(idx * std::mem::size_of::<T>()) as *mut u32 }
    }

    /// a Hal method wrote this buffer's device memory; `root`: hash_fold wrote a node heap's
    /// root layer, so the heap's host mirror starts copying
    fn written(&self, root: bool) {
        let a = self.alloc.borrow();
        if root {
            a.mirror_start();
        } else {
            a.written();
        }
    }

    fn read(&self, offset: usize, len: usize) -> Vec<T> {
        let mut out = Vec::<T>::with_capacity(len);
        let bytes = len * std::mem::size_of::<T>();
        if let Some(g) = self.alloc.borrow().gathered.borrow().as_ref() {
            let at = (self.offset + offset) * std::mem::size_of::<T>();
            unsafe {
                std::ptr::copy_nonoverlapping((g.as_ptr() as *const u8).add(at), out.as_mut_ptr() as *mut u8, bytes);
                out.set_len(len);
            }
            return out;
        }
        if bytes > 0 {
            check(unsafe { r0hip_memcpy_d2h(out.as_mut_ptr() as *mut c_void, self.dev_at(offset) as *const c_void, bytes) });
        }
        unsafe { out.set_len(len) };
        out
    }
}

impl<T: Clone> Buffer<T> for BufferImpl<T> {
    fn name(&self) -> &'static str {
        self.alloc.borrow().name
    }

    fn size(&self) -> usize {
        self.size
    }

    fn slice(&self, offset: usize, size: usize) -> Self {
        assert!(offset + size <= self.size, "slice [{offset}, {}) of {}", offset + size, self.size);
        Self { alloc: self.alloc.clone(), offset: self.offset + offset, size, _t: PhantomData }
    }

    fn get_at(&self, idx: usize) -> T {
        assert!(idx < self.size);
        let a = self.alloc.borrow();
        if let Some(h) = a.host() {
            let at = (self.offset + idx) * std::mem::size_of::<T>();
            return unsafe { std::ptr::read_unaligned(h.add(at) as *const T) };
        }
        drop(a);
        self.read(idx, 1).pop().unwrap()
    }

    fn view<F: FnOnce(&[T])>(&self, f: F) {
        scope!("view");
        f(&self.read(0, self.size));
    }

    fn view_mut<F: FnOnce(&mut [T])>(&self, f: F) {
        scope!("view_mut");
        let mut host = self.read(0, self.size);
        f(&mut host);
        self.written(false);
        let bytes = std::mem::size_of_val(host.as_slice());
        if bytes > 0 {
            check(unsafe { r0hip_memcpy_h2d(self.dev_void(), host.as_ptr() as *const c_void, bytes) });
        }
    }

    fn to_vec(&self) -> Vec<T> {
        self.read(0, self.size)
    }
}

// ---------------------------------------------------------------------------------------
// Hash suites: the device hashing is selected by a suite number, the host side (transcript
// RNG, header and coefficient hashes) is the CPU HashSuite, as in cuda.rs:89-233.

pub trait HipHash {
    const SUITE: i32;
    fn new_suite() -> HashSuite<BabyBear>;
}

pub struct HipHashPoseidon2;
pub struct HipHashSha256;
pub struct HipHashPoseidon254;

impl HipHash for HipHashPoseidon2 {
    const SUITE: i32 = R0HIP_POSEIDON2;
    fn new_suite() -> HashSuite<BabyBear> {
        Poseidon2HashSuite::new_suite()
    }
}

impl HipHash for HipHashSha256 {
    const SUITE: i32 = R0HIP_SHA256;
    fn new_suite() -> HashSuite<BabyBear> {
        Sha256HashSuite::new_suite()
    }
}

impl HipHash for HipHashPoseidon254 {
    const SUITE: i32 = R0HIP_POSEIDON254;
    fn new_suite() -> HashSuite<BabyBear> {
        Poseidon254HashSuite::new_suite()
    }
}

// ---------------------------------------------------------------------------------------
// The HAL

pub struct HipHal<HS: HipHash> {
    suite: HashSuite<BabyBear>,
    _lock: ReentrantMutexGuard<'static, ()>,
    _hs: PhantomData<HS>,
}

pub type HipHalPoseidon2 = HipHal<HipHashPoseidon2>;
pub type HipHalSha256 = HipHal<HipHashSha256>;
pub type HipHalPoseidon254 = HipHal<HipHashPoseidon254>;

impl<HS: HipHash> Default for HipHal<HS> {
    fn default() -> Self {
        Self::new()
    }
}

impl<HS: HipHash> HipHal<HS> {
    pub fn new() -> Self {
        let _lock = device_lock().lock();
        check(unsafe { r0hip_init(device_ordinal()) });
        Self { suite: HS::new_suite(), _lock, _hs: PhantomData }
    }

    /// Name and memory of the bound device (for logs; cust's Device::name role).
    pub fn device_info(&self) -> (String, u64) {
        let mut name = [0 as std::os::raw::c_char; 256];
        let mut mem = 0u64;
        check(unsafe { r0hip_device_info(name.as_mut_ptr(), name.len(), &mut mem) });
        (unsafe { CStr::from_ptr(name.as_ptr()) }.to_string_lossy().into_owned(), mem)
    }
}

fn words<E: Elem>(v: &[E]) -> Vec<u32> {
    v.iter().flat_map(|e| e.to_u32_words()).collect()
}

fn lg(n: usize) -> u32 {
    let l = log2_ceil(n);
    assert_eq!(1 << l, n, "{n} is not a power of two");
    l as u32
}

impl<HS: HipHash> Hal for HipHal<HS> {
    type Field = BabyBear;
    type Elem = BabyBearElem;
    type ExtElem = BabyBearExtElem;
    type Buffer<T: Clone + std::fmt::Debug + PartialEq> = BufferImpl<T>;

    fn has_unified_memory(&self) -> bool {
        false
    }

    fn get_hash_suite(&self) -> &HashSuite<Self::Field> {
        &self.suite
    }

    fn alloc_digest(&self, name: &'static str, size: usize) -> Self::Buffer<Digest> {
        BufferImpl::new(name, size)
    }

    fn alloc_elem(&self, name: &'static str, size: usize) -> Self::Buffer<Self::Elem> {
        BufferImpl::new(name, size)
    }

    fn alloc_extelem(&self, name: &'static str, size: usize) -> Self::Buffer<Self::ExtElem> {
        BufferImpl::new(name, size)
    }

    fn alloc_u32(&self, name: &'static str, size: usize) -> Self::Buffer<u32> {
        BufferImpl::new(name, size)
    }

    // device-side fills instead of the trait's view_mut round trip (hal/mod.rs:72-98)
    fn alloc_elem_init(&self, name: &'static str, size: usize, value: Self::Elem) -> Self::Buffer<Self::Elem> {
        let buf = self.alloc_elem(name, size);
        check(unsafe { r0hip_memset32(buf.dev_void(), value.to_u32_words()[0], size) });
        buf
    }

    fn alloc_extelem_zeroed(&self, name: &'static str, size: usize) -> Self::Buffer<Self::ExtElem> {
        let buf = self.alloc_extelem(name, size);
        check(unsafe { r0hip_memset32(buf.dev_void(), 0, size * BabyBearExtElem::EXT_SIZE) });
        buf
    }

    fn copy_from_digest(&self, name: &'static str, slice: &[Digest]) -> Self::Buffer<Digest> {
        BufferImpl::from_slice(name, slice)
    }

    fn copy_from_elem(&self, name: &'static str, slice: &[Self::Elem]) -> Self::Buffer<Self::Elem> {
        BufferImpl::from_slice(name, slice)
    }

    fn copy_from_extelem(&self, name: &'static str, slice: &[Self::ExtElem]) -> Self::Buffer<Self::ExtElem> {
        BufferImpl::from_slice(name, slice)
    }

    fn copy_from_u32(&self, name: &'static str, slice: &[u32]) -> Self::Buffer<u32> {
        BufferImpl::from_slice(name, slice)
    }

    fn batch_expand_into_evaluate_ntt(
        &self,
        output: &Self::Buffer<Self::Elem>,
        input: &Self::Buffer<Self::Elem>,
        count: usize,
        expand_bits: usize,
    ) {
        assert_eq!(output.size() % count, 0);
        assert_eq!(input.size() * (1 << expand_bits), output.size());
        let lg_out = lg(output.size() / count);
        check(unsafe { r0hip_batch_expand_into_evaluate_ntt(output.dev(), input.dev(), count, lg_out, expand_bits as u32) });
    }

    fn batch_interpolate_ntt(&self, io: &Self::Buffer<Self::Elem>, count: usize) {
        assert_eq!(io.size() % count, 0);
        check(unsafe { r0hip_batch_interpolate_ntt(io.dev(), count, lg(io.size() / count)) });
    }

    fn batch_bit_reverse(&self, io: &Self::Buffer<Self::Elem>, count: usize) {
        assert_eq!(io.size() % count, 0);
        check(unsafe { r0hip_batch_bit_reverse(io.dev(), count, lg(io.size() / count)) });
    }

    fn batch_evaluate_any(
        &self,
        coeffs: &Self::Buffer<Self::Elem>,
        poly_count: usize,
        which: &Self::Buffer<u32>,
        xs: &Self::Buffer<Self::ExtElem>,
        out: &Self::Buffer<Self::ExtElem>,
    ) {
        assert_eq!(which.size(), xs.size());
        assert_eq!(which.size(), out.size());
        let lg_size = lg(coeffs.size() / poly_count);
        check(unsafe {
            r0hip_batch_evaluate_any(out.dev(), coeffs.dev(), poly_count, lg_size, which.dev(), xs.dev(), which.size())
        });
    }

    fn zk_shift(&self, io: &Self::Buffer<Self::Elem>, count: usize) {
        assert_eq!(io.size() % count, 0);
        check(unsafe { r0hip_zk_shift(io.dev(), count, lg(io.size() / count)) });
    }

    fn mix_poly_coeffs(
        &self,
        out: &Self::Buffer<Self::ExtElem>,
        mix_start: &Self::ExtElem,
        mix: &Self::ExtElem,
        input: &Self::Buffer<Self::Elem>,
        combos: &Self::Buffer<u32>,
        input_size: usize,
        count: usize,
    ) {
        assert_eq!(input.size(), input_size * count);
        assert_eq!(combos.size(), input_size);
        // the combo ids are read on the host to group the columns per combo
        let ids = combos.to_vec();
        let (start, m) = (mix_start.to_u32_words(), mix.to_u32_words());
        check(unsafe {
            r0hip_mix_poly_coeffs(out.dev(), input.dev(), ids.as_ptr(), start.as_ptr(), m.as_ptr(), input_size, count)
        });
    }

    fn eltwise_add_elem(
        &self,
        output: &Self::Buffer<Self::Elem>,
        input1: &Self::Buffer<Self::Elem>,
        input2: &Self::Buffer<Self::Elem>,
    ) {
        assert_eq!(output.size(), input1.size());
        assert_eq!(output.size(), input2.size());
        check(unsafe { r0hip_eltwise_add_elem(output.dev(), input1.dev(), input2.dev(), output.size()) });
    }

    fn eltwise_sum_extelem(&self, output: &Self::Buffer<Self::Elem>, input: &Self::Buffer<Self::ExtElem>) {
        let count = output.size() / BabyBearExtElem::EXT_SIZE;
        assert_eq!(input.size() % count, 0);
        check(unsafe { r0hip_eltwise_sum_extelem(output.dev(), input.dev(), input.size() / count, count) });
    }

    fn eltwise_copy_elem(&self, output: &Self::Buffer<Self::Elem>, input: &Self::Buffer<Self::Elem>) {
        assert_eq!(output.size(), input.size());
        check(unsafe { r0hip_eltwise_copy_elem(output.dev(), input.dev(), output.size()) });
    }

    fn eltwise_copy_elem_slice(
        &self,
        into: &Self::Buffer<Self::Elem>,
        from: &[Self::Elem],
        from_rows: usize,
        from_cols: usize,
        from_offset: usize,
        from_stride: usize,
        into_offset: usize,
        into_stride: usize,
    ) {
        let staged = self.copy_from_elem("from", from);
        check(unsafe {
            r0hip_eltwise_copy_elem_slice(
                into.dev(),
                staged.dev(),
                from_rows,
                from_cols,
                from_offset,
                from_stride,
                into_offset,
                into_stride,
            )
        });
    }

    fn eltwise_zeroize_elem(&self, elems: &Self::Buffer<Self::Elem>) {
        check(unsafe { r0hip_eltwise_zeroize_elem(elems.dev(), elems.size()) });
    }

    fn fri_fold(&self, output: &Self::Buffer<Self::Elem>, input: &Self::Buffer<Self::Elem>, mix: &Self::ExtElem) {
        let count = output.size() / BabyBearExtElem::EXT_SIZE;
        assert_eq!(input.size(), output.size() * crate::FRI_FOLD);
        let m = mix.to_u32_words();
        check(unsafe { r0hip_fri_fold(output.dev(), input.dev(), m.as_ptr(), count) });
    }

    fn hash_rows(&self, output: &Self::Buffer<Digest>, matrix: &Self::Buffer<Self::Elem>) {
        let rows = output.size();
        assert_eq!(matrix.size() % rows, 0);
        check(unsafe { r0hip_hash_rows(HS::SUITE, output.dev(), matrix.dev(), rows, matrix.size() / rows) });
        output.written(false);
    }

    fn hash_fold(&self, io: &Self::Buffer<Digest>, input_size: usize, output_size: usize) {
        assert_eq!(input_size, 2 * output_size);
        check(unsafe { r0hip_hash_fold(HS::SUITE, io.dev(), input_size, output_size) });
        io.written(output_size == 1);
    }

    fn gather_sample(
        &self,
        dst: &Self::Buffer<Self::Elem>,
        src: &Self::Buffer<Self::Elem>,
        idx: usize,
        size: usize,
        stride: usize,
    ) {
        assert!(dst.size() >= size);
        {
            // a fresh whole-allocation destination: gather straight to the host (it is read back
            // before any device use in MerkleTreeProver::prove; `device` uploads it otherwise)
            let a = dst.alloc.borrow();
            if a.ptr.get().is_null() && dst.offset == 0 && size * 4 == a.bytes {
                let mut g = vec![0u32; size];
                check(unsafe { r0hip_gather_sample_host(g.as_mut_ptr(), src.dev(), idx, size, stride) });
                *a.gathered.borrow_mut() = Some(g);
                return;
            }
        }
        check(unsafe { r0hip_gather_sample(dst.dev(), src.dev(), idx, size, stride) });
    }

    fn scatter(&self, into: &Self::Buffer<Self::Elem>, index: &[u32], offsets: &[u32], values: &[Self::Elem]) {
        if index.is_empty() {
            return;
        }
        let (di, doff, dv) = (
            self.copy_from_u32("index", index),
            self.copy_from_u32("offsets", offsets),
            self.copy_from_elem("values", values),
        );
        check(unsafe { r0hip_scatter(into.dev(), di.dev(), doff.dev(), dv.dev(), index.len() - 1) });
    }

    fn prefix_products(&self, io: &Self::Buffer<Self::ExtElem>) {
        check(unsafe { r0hip_prefix_products(io.dev(), io.size()) });
    }

    fn combos_prepare(
        &self,
        combos: &Self::Buffer<Self::ExtElem>,
        coeff_u: &[Self::ExtElem],
        combo_count: usize,
        cycles: usize,
        reg_sizes: &[u32],
        reg_combo_ids: &[u32],
        mix: &Self::ExtElem,
    ) {
        scope!("combos_prepare");
        assert_eq!(reg_sizes.len(), reg_combo_ids.len());
        let (u, m) = (words(coeff_u), mix.to_u32_words());
        check(unsafe {
            r0hip_combos_prepare(
                combos.dev(),
                u.as_ptr(),
                combo_count,
                cycles,
                reg_sizes.as_ptr(),
                reg_combo_ids.as_ptr(),
                reg_sizes.len(),
                m.as_ptr(),
            )
        });
    }

    fn combos_divide(
        &self,
        combos: &Self::Buffer<Self::ExtElem>,
        chunks: Vec<(usize, Vec<Self::ExtElem>)>,
        cycles: usize,
    ) {
        scope!("combos_divide");
        // chunk i covers combos[i * cycles ..]; the Prover hands them over in order
        let mut pows = Vec::new();
        let mut begin = vec![0u32];
        for (n, (i, zs)) in chunks.iter().enumerate() {
            assert_eq!(*i, n, "combos_divide: chunks out of order");
            pows.extend(words(zs));
            begin.push((pows.len() / BabyBearExtElem::EXT_SIZE) as u32);
        }
        let mut bad = -1i64;
        check(unsafe {
            r0hip_combos_divide(combos.dev(), chunks.len(), pows.as_ptr(), begin.as_ptr(), cycles, &mut bad)
        });
        assert_eq!(bad, -1, "combos_divide: nonzero remainder in chunk {bad}");
    }
}

impl<HS: HipHash> HipHal<HS> {
    /// supra_poly_divide's role (cuda.rs:424-449): in-place division of one FpExt polynomial
    /// by (x - z), returning the remainder.
    pub fn poly_divide(&self, poly: &BufferImpl<BabyBearExtElem>, z: BabyBearExtElem) -> BabyBearExtElem {
        let mut rem = [0u32; 4];
        let zw = z.to_u32_words();
        check(unsafe { r0hip_poly_divide(poly.dev(), poly.size(), rem.as_mut_ptr(), zw.as_ptr()) });
        BabyBearExtElem::from_u32_words(&rem)
    }

    /// Peak device bytes of the HAL's buffers since the last reset (libr0hip's own
    /// accounting; the Rust MemoryTracker above counts the same allocations).
    pub fn peak_device_bytes(&self) -> u64 {
        let mut s = [0u64; 5];
        check(unsafe { r0hip_mem_stats(s.as_mut_ptr()) });
        s[1]
    }
}

// The CPU-vs-device checks of hal/testutil.rs, as cuda.rs:1050-1137 instantiates them.
#[cfg(test)]
mod tests {
    use test_log::test;

    use super::{HipHalPoseidon2, HipHalPoseidon254, HipHalSha256};
    use crate::hal::testutil;

    #[test]
    #[should_panic]
    fn check_req() {
        testutil::check_req(HipHalSha256::new());
    }

    #[test]
    fn eltwise_add_elem() {
        testutil::eltwise_add_elem(HipHalSha256::new());
    }

    #[test]
    fn eltwise_copy_elem() {
        testutil::eltwise_copy_elem(HipHalSha256::new());
    }

    #[test]
    fn eltwise_sum_extelem() {
        testutil::eltwise_sum_extelem(HipHalSha256::new());
    }

    #[test]
    fn hash_rows_sha256() {
        testutil::hash_rows(HipHalSha256::new());
    }

    #[test]
    fn hash_fold_sha256() {
        testutil::hash_fold(HipHalSha256::new());
    }

    #[test]
    fn hash_rows_poseidon2() {
        testutil::hash_rows(HipHalPoseidon2::new());
    }

    #[test]
    fn hash_fold_poseidon2() {
        testutil::hash_fold(HipHalPoseidon2::new());
    }

    #[test]
    fn hash_rows_poseidon254() {
        testutil::hash_rows(HipHalPoseidon254::new());
    }

    #[test]
    fn hash_fold_poseidon254() {
        testutil::hash_fold(HipHalPoseidon254::new());
    }

    #[test]
    fn fri_fold() {
        testutil::fri_fold(HipHalSha256::new());
    }

    #[test]
    fn batch_expand_into_evaluate_ntt() {
        testutil::batch_expand_into_evaluate_ntt(HipHalSha256::new());
    }

    #[test]
    fn batch_interpolate_ntt() {
        testutil::batch_interpolate_ntt(HipHalSha256::new());
    }

    #[test]
    fn batch_bit_reverse() {
        testutil::batch_bit_reverse(HipHalSha256::new());
    }

    #[test]
    fn batch_evaluate_any() {
        testutil::batch_evaluate_any(HipHalSha256::new());
    }

    #[test]
    fn gather_sample() {
        testutil::gather_sample(HipHalSha256::new());
    }

    #[test]
    fn zk_shift() {
        testutil::zk_shift(HipHalSha256::new());
    }

    #[test]
    fn mix_poly_coeffs() {
        testutil::mix_poly_coeffs(HipHalSha256::new());
    }
}
