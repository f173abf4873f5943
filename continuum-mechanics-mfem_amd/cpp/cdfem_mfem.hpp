// cdfem_mfem.hpp — MFEM-shaped C++ host API over the cdfem C-ABI (include/cdfem.h).
//
// The host side of the drop-in boundary: the classes and member functions the
// reference driver myapps/convection_diffusion/linear_convection_diffusion_2D.cpp calls on its hot
// path, with MFEM's names, argument meaning and ownership rules, backed by the MI355X kernels:
//
//   reference call (file:line)                               here
//   ParMesh / Mesh::MakeCartesian*  (:300)                   Mesh::MakeCartesian2D / 3D
//   H1_FECollection, ParFiniteElementSpace (:311-313)        H1_FECollection, FiniteElementSpace
//   GetEssentialTrueDofs(ess_bdr, list) (:319-322)           FiniteElementSpace::GetEssentialTrueDofs
//   Coefficient::Eval(T, ip), T.Transform(ip, x) (:165-205)  Coefficient, ElementTransformation
//   ConstantCoefficient / VectorConstantCoefficient (:331-333)
//   ParBilinearForm + Diffusion/Convection/MassIntegrator,   BilinearForm (partial assembly on the
//     AddDomainIntegrator (owns), Assemble (:335-339)          GPU; integrators owned by the form)
//   ParLinearForm + DomainLFIntegrator, Assemble (:341-343)  LinearForm, DomainLFIntegrator
//   ParGridFunction, ProjectBdrCoefficient (:345-347)        GridFunction
//   FormLinearSystem(ess, u, b, A, X, B) (:349-351)          BilinearForm::FormLinearSystem
//   PetscParMatrix + PetscLinearSolver (:364-374)            PetscParMatrix, PetscLinearSolver (the
//     options of Input/petsc.opts via MFEMInitializePetsc)   GPU GMRES/CG, same option keys)
//   CGSolver (mesh_recession_handler.cpp:270-276)            CGSolver
//   RecoverFEMSolution (:377), ComputeL2Error (:383-392)     BilinearForm / GridFunction
//
// Error behaviour: every failing C-ABI call throws std::runtime_error carrying cdfem_last_error
// (the reference drivers catch std::exception at main and return 3, :435-442); MFEM_VERIFY-style
// misuse (wrong sizes) throws std::invalid_argument.  There is no CPU fallback: constructing a
// form without a GPU throws.
//
// Scope (single rank): L-vector == T-vector (P = identity), so RecoverFEMSolution copies X into x.
// The multi-GPU slab path is driven through the C-ABI (cdfem_comm_* / cdfem_set_slab).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "cdfem.h"

namespace cdfem {
namespace mfem {

using real_t = double;

inline void check(int rc, const cdfem_ctx *ctx, const char *what)
{
    if (rc == CDFEM_OK) return;
    std::string msg = std::string(what) + " failed (status " + std::to_string(rc) + ")";
    if (ctx) msg += ": " + std::string(cdfem_last_error(ctx));
    throw std::runtime_error(msg);
}

// ---- containers ---------------------------------------------------------------------------------
class Vector {
public:
    Vector() = default;
    explicit Vector(int n) : d_((size_t)n, 0.0) {}
    int Size() const { return (int)d_.size(); }
    void SetSize(int n) { d_.assign((size_t)n, 0.0); }
    double *GetData() { return d_.data(); }
    const double *GetData() const { return d_.data(); }
    double &operator[](int i) { return d_[(size_t)i]; }
    double operator[](int i) const { return d_[(size_t)i]; }
    double &operator()(int i) { return d_[(size_t)i]; }
    double operator()(int i) const { return d_[(size_t)i]; }
    Vector &operator=(double v)
    {
        std::fill(d_.begin(), d_.end(), v);
        return *this;
    }
    double operator*(const Vector &o) const
    {
        double s = 0.0;
        for (size_t i = 0; i < d_.size(); ++i) s += d_[i] * o.d_[i];
        return s;
    }
    double Norml2() const { return std::sqrt((*this) * (*this)); }
    double Normlinf() const
    {
        double m = 0.0;
        for (double v : d_) m = std::max(m, std::fabs(v));
        return m;
    }
    void Add(double a, const Vector &x)
    {
        for (size_t i = 0; i < d_.size(); ++i) d_[i] += a * x.d_[i];
    }

private:
    std::vector<double> d_;
};

template <class T>
class Array {
public:
    Array() = default;
    explicit Array(int n) : d_((size_t)n) {}
    int Size() const { return (int)d_.size(); }
    void SetSize(int n) { d_.resize((size_t)n); }
    void Append(const T &v) { d_.push_back(v); }
    T &operator[](int i) { return d_[(size_t)i]; }
    const T &operator[](int i) const { return d_[(size_t)i]; }
    Array &operator=(const T &v)
    {
        std::fill(d_.begin(), d_.end(), v);
        return *this;
    }
    T Max() const { return d_.empty() ? T() : *std::max_element(d_.begin(), d_.end()); }
    T *GetData() { return d_.data(); }
    const T *GetData() const { return d_.data(); }
    bool operator==(const Array &o) const { return d_ == o.d_; }

private:
    std::vector<T> d_;
};

// ---- geometry / quadrature -----------------------------------------------------------------------
struct IntegrationPoint {
    double x = 0.0, y = 0.0, z = 0.0, weight = 0.0;
};

struct Geometry {
    enum Type { SQUARE = 3, CUBE = 5 };
    static constexpr int NumGeom = 8;
};

// Tensor Gauss-Legendre rule exact for polynomials of the given order (MFEM IntRules.Get on
// SQUARE / CUBE: n = order / 2 + 1 points per direction).
class IntegrationRule {
public:
    IntegrationRule() = default;
    IntegrationRule(int geom, int order) : geom_(geom), order_(order) {}
    int GetOrder() const { return order_; }
    int Points1D() const { return order_ / 2 + 1; }

private:
    int geom_ = Geometry::SQUARE, order_ = 2;
};

class IntegrationRules {
public:
    const IntegrationRule &Get(int geom, int order)
    {
        const int key = geom * 1024 + order;
        auto it = rules_.find(key);
        if (it == rules_.end()) it = rules_.emplace(key, IntegrationRule(geom, order)).first;
        return it->second;
    }

private:
    std::map<int, IntegrationRule> rules_;
};
inline IntegrationRules IntRules;

// The physical point of the quadrature point being sampled; user coefficients call
// T.Transform(ip, x) exactly as in the reference (linear_convection_diffusion_2D.cpp:166-168).
class ElementTransformation {
public:
    int ElementNo = -1;
    int Attribute = 1;
    void Transform(const IntegrationPoint &, Vector &x) const
    {
        x.SetSize(dim_);
        for (int k = 0; k < dim_; ++k) x[k] = X_[k];
    }
    void SetPoint(int dim, const double *X)
    {
        dim_ = dim;
        for (int k = 0; k < dim; ++k) X_[k] = X[k];
    }

private:
    int dim_ = 0;
    double X_[3] = {0, 0, 0};
};

// ---- coefficients --------------------------------------------------------------------------------
class Coefficient {
public:
    virtual ~Coefficient() = default;
    virtual real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) = 0;
    virtual void SetTime(double t) { time = t; }
    double GetTime() const { return time; }

protected:
    double time = 0.0;
};

class ConstantCoefficient : public Coefficient {
public:
    double constant;
    explicit ConstantCoefficient(double c = 1.0) : constant(c) {}
    real_t Eval(ElementTransformation &, const IntegrationPoint &) override { return constant; }
};

class FunctionCoefficient : public Coefficient {
public:
    explicit FunctionCoefficient(std::function<double(const Vector &)> f) : f_(std::move(f)) {}
    explicit FunctionCoefficient(std::function<double(const Vector &, double)> ft) : ft_(std::move(ft)) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        return f_ ? f_(x) : ft_(x, time);
    }

private:
    std::function<double(const Vector &)> f_;
    std::function<double(const Vector &, double)> ft_;
};

class VectorCoefficient {
public:
    explicit VectorCoefficient(int vd) : vdim(vd) {}
    virtual ~VectorCoefficient() = default;
    int GetVDim() const { return vdim; }
    virtual void Eval(Vector &V, ElementTransformation &T, const IntegrationPoint &ip) = 0;
    virtual void SetTime(double t) { time = t; }

protected:
    int vdim;
    double time = 0.0;
};

class VectorConstantCoefficient : public VectorCoefficient {
public:
    explicit VectorConstantCoefficient(const Vector &v) : VectorCoefficient(v.Size()), vec(v) {}
    void Eval(Vector &V, ElementTransformation &, const IntegrationPoint &) override { V = vec; }
    const Vector &GetVec() const { return vec; }

private:
    Vector vec;
};

class VectorFunctionCoefficient : public VectorCoefficient {
public:
    VectorFunctionCoefficient(int dim, std::function<void(const Vector &, Vector &)> f)
        : VectorCoefficient(dim), f_(std::move(f)) {}
    void Eval(Vector &V, ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        V.SetSize(vdim);
        f_(x, V);
    }

private:
    std::function<void(const Vector &, Vector &)> f_;
};

// ---- mesh and H1 space ------------------------------------------------------------------------
struct Element {
    enum Type { QUADRILATERAL = 3, HEXAHEDRON = 5 };
};

// Structured box [0,sx] x [0,sy] (x [0,sz]).  Boundary attributes follow MFEM's Cartesian
// convention: 2D 1 bottom (y=0), 2 right (x=sx), 3 top, 4 left; 3D 1 z=0, 2 y=0, 3 x=sx, 4 y=sy,
// 5 x=0, 6 z=sz.
class Mesh {
public:
    // gmsh v2.2 simplex mesh file, as Mesh(mesh_file, 1, 1) at linear_convection_diffusion_2D.cpp:290
    explicit Mesh(const char *path, int = 1, int = 1) : dim_(0), n_{0, 0, 0}, s_{1.0, 1.0, 1.0}, path_(path)
    {
        int ne = 0;
        int64_t nl = 0;
        check(cdfem_gmsh_sizes(path, 1, &dim_, &ne, &nl), nullptr, "cdfem_gmsh_sizes (mesh file)");
        ne_ = ne;
        std::vector<int32_t> mask((size_t)nl);
        check(cdfem_gmsh_mesh(path, 1, nullptr, nullptr, mask.data(), nullptr), nullptr, "cdfem_gmsh_mesh");
        int32_t all = 0;
        for (int32_t m : mask) all |= m;
        for (int a = 1; a <= 31; ++a)
            if (all & (1 << (a - 1))) bdr_attributes.Append(a);
    }
    bool FromFile() const { return !path_.empty(); }
    const std::string &Path() const { return path_; }
    static Mesh MakeCartesian2D(int nx, int ny, Element::Type, bool = false, double sx = 1.0, double sy = 1.0)
    {
        return Mesh(2, nx, ny, 1, sx, sy, 1.0);
    }
    static Mesh MakeCartesian3D(int nx, int ny, int nz, Element::Type, double sx = 1.0, double sy = 1.0,
                                double sz = 1.0)
    {
        return Mesh(3, nx, ny, nz, sx, sy, sz);
    }
    int Dimension() const { return dim_; }
    int GetNE() const { return FromFile() ? ne_ : dim_ == 3 ? n_[0] * n_[1] * n_[2] : n_[0] * n_[1]; }
    int N(int k) const { return n_[k]; }
    double Size(int k) const { return s_[k]; }
    Array<int> bdr_attributes;

private:
    Mesh(int dim, int nx, int ny, int nz, double sx, double sy, double sz)
        : dim_(dim), n_{nx, ny, nz}, s_{sx, sy, sz}
    {
        if (nx < 1 || ny < 1 || nz < 1) throw std::invalid_argument("Mesh: element counts must be >= 1");
        for (int a = 1; a <= 2 * dim; ++a) bdr_attributes.Append(a);
    }
    int dim_;
    int n_[3];
    double s_[3];
    std::string path_;
    int ne_ = 0;
};
using ParMesh = Mesh;

class H1_FECollection {
public:
    H1_FECollection(int p, int dim) : p_(p), dim_(dim)
    {
        if (p < 1) throw std::invalid_argument("H1_FECollection: order must be >= 1");
    }
    int GetOrder() const { return p_; }
    int GetDim() const { return dim_; }

private:
    int p_, dim_;
};

class DeviceSpace;

class FiniteElementSpace {
public:
    FiniteElementSpace(Mesh *mesh, H1_FECollection *fec) : mesh_(mesh), fec_(fec)
    {
        if (mesh->Dimension() != fec->GetDim()) throw std::invalid_argument("FiniteElementSpace: dim mismatch");
        const int dim = mesh->Dimension(), p = fec->GetOrder();
        if (mesh->FromFile()) {  // simplices: numbering and boundary attributes from the reader
            int d = 0;
            int64_t nl = 0;
            check(cdfem_gmsh_sizes(mesh->Path().c_str(), p, &d, &ne_, &nl), nullptr, "cdfem_gmsh_sizes");
            nl_ = (int)nl;
            nv_ = dim + 1;
            nd_ = p == 1 ? dim + 1 : p == 2 ? (dim + 1) * (dim + 2) / 2 : 10;
            verts_.resize((size_t)ne_ * nv_ * dim);
            dofs_.resize((size_t)ne_ * nd_);
            xyz_.resize((size_t)nl_ * dim);
            bmask_.resize(nl_);
            check(cdfem_gmsh_mesh(mesh->Path().c_str(), p, verts_.data(), dofs_.data(), bmask_.data(), xyz_.data()),
                  nullptr, "cdfem_gmsh_mesh");
            simplex_ = true;
            return;
        }
        int64_t nl = 0;
        int ness = 0;
        check(cdfem_box_sizes(dim, mesh->N(0), mesh->N(1), mesh->N(2), p, 0, 0, &ne_, &nl, &ness), nullptr,
              "cdfem_box_sizes");
        nl_ = (int)nl;
        nv_ = 1 << dim;
        nd_ = dim == 3 ? (p + 1) * (p + 1) * (p + 1) : (p + 1) * (p + 1);
        verts_.resize((size_t)ne_ * nv_ * dim);
        dofs_.resize((size_t)ne_ * nd_);
        std::vector<int32_t> ess((size_t)ness);
        xyz_.resize((size_t)nl_ * dim);
        check(cdfem_box_mesh(dim, mesh->N(0), mesh->N(1), mesh->N(2), p, 0, 0, 0.0, verts_.data(), dofs_.data(),
                             ess.data(), xyz_.data()),
              nullptr, "cdfem_box_mesh");
        for (size_t i = 0; i < verts_.size(); ++i) verts_[i] *= mesh->Size((int)(i % dim));
        for (size_t i = 0; i < xyz_.size(); ++i) xyz_[i] *= mesh->Size((int)(i % dim));
    }
    Mesh *GetMesh() const { return mesh_; }
    int GetOrder() const { return fec_->GetOrder(); }
    int GetVSize() const { return nl_; }
    int GetTrueVSize() const { return nl_; }
    int TrueVSize() const { return nl_; }
    int GetNE() const { return ne_; }

    // dofs on the boundary faces whose attribute is marked (ess_bdr[attr - 1] != 0)
    void GetEssentialTrueDofs(const Array<int> &ess_bdr, Array<int> &list) const
    {
        const int dim = mesh_->Dimension();
        list.SetSize(0);
        for (int i = 0; i < nl_; ++i)
            if (OnMarkedBoundary(i, ess_bdr, dim)) list.Append(i);
    }
    bool OnMarkedBoundary(int i, const Array<int> &marker, int dim) const
    {
        if (simplex_) {
            for (int a = 1; a <= marker.Size() && a <= 31; ++a)
                if (marker[a - 1] && (bmask_[i] & (1 << (a - 1)))) return true;
            return false;
        }
        const double *X = &xyz_[(size_t)i * dim];
        auto at = [&](int attr) { return attr <= marker.Size() && marker[attr - 1] != 0; };
        const double sx = mesh_->Size(0), sy = mesh_->Size(1), sz = mesh_->Size(2);
        if (dim == 2)
            return (X[1] == 0.0 && at(1)) || (X[0] == sx && at(2)) || (X[1] == sy && at(3)) || (X[0] == 0.0 && at(4));
        return (X[2] == 0.0 && at(1)) || (X[1] == 0.0 && at(2)) || (X[0] == sx && at(3)) || (X[1] == sy && at(4)) ||
               (X[0] == 0.0 && at(5)) || (X[2] == sz && at(6));
    }
    const std::vector<double> &ElementVertices() const { return verts_; }
    const std::vector<int32_t> &ElementDofs() const { return dofs_; }
    const std::vector<double> &DofCoordinates() const { return xyz_; }
    bool Simplex() const { return simplex_; }
    int NumElementDofs() const { return nd_; }
    // device context for linear forms on this space, created on first use and reused (the
    // reference builds a new ParLinearForm every time step, diffusion_mms.cpp:434-437)
    std::shared_ptr<DeviceSpace> &LinearFormDevice() const { return lf_dev_; }

private:
    mutable std::shared_ptr<DeviceSpace> lf_dev_;
    Mesh *mesh_;
    H1_FECollection *fec_;
    int ne_ = 0, nl_ = 0, nv_ = 0, nd_ = 0;
    bool simplex_ = false;
    std::vector<double> verts_, xyz_;
    std::vector<int32_t> dofs_, bmask_;
};
using ParFiniteElementSpace = FiniteElementSpace;

// ---- device context per form (one cdfem_ctx: mesh + operator resident in HBM) -------------------
class DeviceSpace {
public:
    explicit DeviceSpace(const FiniteElementSpace &fes, const Array<int> &ess, bool structured = true)
    {
        const char *dev = std::getenv("CDFEM_DEVICE");
        check(cdfem_create(dev ? std::atoi(dev) : 0, &ctx_), nullptr, "cdfem_create (no GPU? there is no CPU path)");
        Upload(fes, ess, structured);
    }
    ~DeviceSpace() { cdfem_destroy(ctx_); }
    DeviceSpace(const DeviceSpace &) = delete;
    DeviceSpace &operator=(const DeviceSpace &) = delete;
    void Upload(const FiniteElementSpace &fes, const Array<int> &ess, bool structured)
    {
        Mesh *m = fes.GetMesh();
        simplex_ = fes.Simplex();
        if (simplex_) {
            check(cdfem_mesh_upload_simplex(ctx_, m->Dimension(), fes.GetOrder(), fes.GetNE(),
                                            fes.ElementVertices().data(), fes.GetVSize(), fes.ElementDofs().data(),
                                            ess.Size(), ess.GetData()),
                  ctx_, "cdfem_mesh_upload_simplex");
            ess_ = ess;
            return;
        }
        check(cdfem_mesh_upload(ctx_, m->Dimension(), fes.GetOrder(), fes.GetNE(), fes.ElementVertices().data(),
                                fes.GetVSize(), fes.ElementDofs().data(), ess.Size(), ess.GetData()),
              ctx_, "cdfem_mesh_upload");
        // the Cartesian box is lexicographic: the structured fast paths (bricks p <= 2, lattice E->L p >= 3)
        if (structured && m->Dimension() == 3)
            check(cdfem_mesh_set_structured(ctx_, m->N(0), m->N(1), m->N(2)), ctx_, "cdfem_mesh_set_structured");
        ess_ = ess;
    }
    cdfem_ctx *ctx() const { return ctx_; }
    const Array<int> &Ess() const { return ess_; }
    bool Simplex() const { return simplex_; }
    // physical coordinates of a rule's points, element-major
    std::vector<double> Points(int rule, int dim, int ne, int &nq) const
    {
        check(cdfem_rule_size(ctx_, rule, &nq), ctx_, "cdfem_rule_size");
        std::vector<double> xyz((size_t)ne * nq * dim);
        check(cdfem_quadrature_points(ctx_, rule, xyz.data(), CDFEM_HOST), ctx_, "cdfem_quadrature_points");
        return xyz;
    }

private:
    cdfem_ctx *ctx_ = nullptr;
    Array<int> ess_;
    bool simplex_ = false;
};

// sample a scalar coefficient at the given points (host virtual calls, as in MFEM)
inline std::vector<double> Sample(Coefficient &q, const std::vector<double> &xyz, int dim, int nq)
{
    ElementTransformation T;
    IntegrationPoint ip;
    const size_t n = xyz.size() / dim;
    std::vector<double> out(n);
    for (size_t i = 0; i < n; ++i) {
        T.ElementNo = (int)(i / nq);
        T.SetPoint(dim, &xyz[i * dim]);
        out[i] = q.Eval(T, ip);
    }
    return out;
}

// ---- operators -----------------------------------------------------------------------------------
class Operator {
public:
    enum Type { ANY_TYPE, Hypre_ParCSR, PETSC_MATAIJ };
    Operator(int h = 0, int w = 0) : height(h), width(w) {}
    virtual ~Operator() = default;
    virtual void Mult(const Vector &x, Vector &y) const = 0;
    int Height() const { return height; }
    int Width() const { return width; }

protected:
    int height, width;
};

class BilinearForm;

// the operator FormLinearSystem returns: ConstrainedOperator(PA) with DIAG_ONE semantics
class ConstrainedPAOperator : public Operator {
public:
    explicit ConstrainedPAOperator(const BilinearForm *a, int n) : Operator(n, n), a_(a) {}
    void Mult(const Vector &x, Vector &y) const override;
    const BilinearForm *Form() const { return a_; }

private:
    const BilinearForm *a_;
};
// the reference casts the FormLinearSystem result to HypreParMatrix (:362): same object here
using HypreParMatrix = ConstrainedPAOperator;

class OperatorHandle {
public:
    OperatorHandle() = default;
    explicit OperatorHandle(Operator::Type t) : type_(t) {}
    void Reset(Operator *op) { op_ = op; }
    Operator *Ptr() const { return op_; }
    Operator *operator->() const { return op_; }
    Operator &operator*() const { return *op_; }
    template <class T>
    T *As() const { return dynamic_cast<T *>(op_); }
    Operator::Type Type() const { return type_; }

private:
    Operator *op_ = nullptr;
    Operator::Type type_ = Operator::ANY_TYPE;
};

// ---- integrators (partial assembly on the GPU) -------------------------------------------------
class BilinearFormIntegrator {
public:
    virtual ~BilinearFormIntegrator() = default;
    virtual unsigned Kind() const = 0;
};

class DiffusionIntegrator : public BilinearFormIntegrator {
public:
    DiffusionIntegrator() : Q_(nullptr) {}
    explicit DiffusionIntegrator(Coefficient &q) : Q_(&q) {}
    unsigned Kind() const override { return CDFEM_DIFFUSION; }
    Coefficient *Q_;
};

class ConvectionIntegrator : public BilinearFormIntegrator {
public:
    explicit ConvectionIntegrator(VectorCoefficient &q, double a = 1.0) : Q_(&q), alpha(a) {}
    unsigned Kind() const override { return CDFEM_CONVECTION; }
    VectorCoefficient *Q_;
    double alpha;
};

class MassIntegrator : public BilinearFormIntegrator {
public:
    MassIntegrator() : Q_(nullptr) {}
    explicit MassIntegrator(Coefficient &q) : Q_(&q) {}
    unsigned Kind() const override { return CDFEM_MASS; }
    Coefficient *Q_;
};

enum class AssemblyLevel { LEGACY, FULL, ELEMENT, PARTIAL, NONE };

class GridFunction;

class BilinearForm : public Operator {
public:
    explicit BilinearForm(FiniteElementSpace *f) : Operator(f->GetVSize(), f->GetVSize()), fes_(f) {}
    // the form takes ownership of the integrator (MFEM semantics, :336-338)
    void AddDomainIntegrator(BilinearFormIntegrator *bfi) { integs_.emplace_back(bfi); }
    void SetAssemblyLevel(AssemblyLevel) {}  // partial assembly on the GPU is the only level
    FiniteElementSpace *FESpace() const { return fes_; }

    void Assemble(int = 1)
    {
        if (!dev_) dev_ = std::make_unique<DeviceSpace>(*fes_, Array<int>());
        Setup();
    }
    void Finalize(int = 1) {}

    // y = A x, unconstrained (BilinearForm::Mult, diffusion_mms.cpp:430)
    void Mult(const Vector &x, Vector &y) const override
    {
        Require(x.Size() == height, "Mult: size");
        y.SetSize(height);
        check(cdfem_pa_mult(ctx(), x.GetData(), y.GetData(), 0, CDFEM_HOST), ctx(), "cdfem_pa_mult");
    }

    // ConstrainedOperator semantics (:349-351): X = x, B = b - A x_e, B[ess] = x[ess]
    void FormLinearSystem(const Array<int> &ess_tdof_list, Vector &x, Vector &b, OperatorHandle &A, Vector &X,
                          Vector &B)
    {
        Require(x.Size() == height && b.Size() == height, "FormLinearSystem: size");
        if (!dev_) throw std::logic_error("FormLinearSystem before Assemble");
        if (!(dev_->Ess() == ess_tdof_list)) {  // the constraint is part of the resident operator
            dev_->Upload(*fes_, ess_tdof_list, true);
            Setup();
        }
        X.SetSize(height);
        B.SetSize(height);
        check(cdfem_form_linear_system(ctx(), x.GetData(), b.GetData(), X.GetData(), B.GetData(), CDFEM_HOST), ctx(),
              "cdfem_form_linear_system");
        cop_ = std::make_unique<ConstrainedPAOperator>(this, height);
        A.Reset(cop_.get());
    }

    // single rank: x = P X with P = I
    void RecoverFEMSolution(const Vector &X, const Vector &, Vector &x) const { x = X; }

    cdfem_ctx *ctx() const { return dev_->ctx(); }

private:
    static void Require(bool ok, const char *what)
    {
        if (!ok) throw std::invalid_argument(what);
    }
    void Setup()
    {
        const int dim = fes_->GetMesh()->Dimension(), ne = fes_->GetNE();
        unsigned kinds = 0;
        double kappa = 0.0, mass = 0.0, alpha = 1.0, conv[3] = {0, 0, 0};
        std::vector<double> kq, mq, cq;
        int nq = 0;
        std::vector<double> xyz;
        auto points = [&]() -> const std::vector<double> & {
            if (xyz.empty()) xyz = dev_->Points(CDFEM_RULE_OPERATOR, dim, ne, nq);
            return xyz;
        };
        auto accumulate = [&](Coefficient *q, double &cst, std::vector<double> &arr) {
            if (!q) {
                cst += 1.0;  // MassIntegrator() / DiffusionIntegrator(): coefficient 1
                if (!arr.empty())
                    for (double &v : arr) v += 1.0;
                return;
            }
            if (auto *c = dynamic_cast<ConstantCoefficient *>(q)) {
                cst += c->constant;
                if (!arr.empty())
                    for (double &v : arr) v += c->constant;
                return;
            }
            std::vector<double> s = Sample(*q, points(), dim, nq);
            if (arr.empty()) arr.assign(s.size(), cst);
            for (size_t i = 0; i < s.size(); ++i) arr[i] += s[i];
        };
        for (auto &bi : integs_) {
            kinds |= bi->Kind();
            if (auto *d = dynamic_cast<DiffusionIntegrator *>(bi.get())) accumulate(d->Q_, kappa, kq);
            else if (auto *m = dynamic_cast<MassIntegrator *>(bi.get())) accumulate(m->Q_, mass, mq);
            else if (auto *c = dynamic_cast<ConvectionIntegrator *>(bi.get())) {
                if (auto *vc = dynamic_cast<VectorConstantCoefficient *>(c->Q_); vc && cq.empty()) {
                    for (int k = 0; k < dim; ++k) conv[k] += c->alpha * vc->GetVec()[k];
                } else {
                    const std::vector<double> &P = points();
                    if (cq.empty()) {
                        cq.resize(P.size());
                        for (size_t i = 0; i < P.size(); ++i) cq[i] = conv[i % dim];
                    }
                    ElementTransformation T;
                    IntegrationPoint ip;
                    Vector V;
                    for (size_t i = 0; i < P.size() / dim; ++i) {
                        T.ElementNo = (int)(i / nq);
                        T.SetPoint(dim, &P[i * dim]);
                        c->Q_->Eval(V, T, ip);
                        for (int k = 0; k < dim; ++k) cq[i * dim + k] += c->alpha * V[k];
                    }
                }
            }
        }
        // hexes / quads: partial assembly; simplices: full assembly (CSR on the GPU)
        auto setup = dev_->Simplex() ? cdfem_fa_setup : cdfem_pa_setup;
        check(setup(ctx(), kinds, kappa, kq.empty() ? nullptr : kq.data(), alpha, conv, cq.empty() ? nullptr : cq.data(),
                    mass, mq.empty() ? nullptr : mq.data()),
              ctx(), dev_->Simplex() ? "cdfem_fa_setup" : "cdfem_pa_setup");
    }

    FiniteElementSpace *fes_;
    std::vector<std::unique_ptr<BilinearFormIntegrator>> integs_;
    std::unique_ptr<DeviceSpace> dev_;
    std::unique_ptr<ConstrainedPAOperator> cop_;
};
using ParBilinearForm = BilinearForm;

inline void ConstrainedPAOperator::Mult(const Vector &x, Vector &y) const
{
    y.SetSize(height);
    check(cdfem_pa_mult(a_->ctx(), x.GetData(), y.GetData(), 1, CDFEM_HOST), a_->ctx(), "cdfem_pa_mult");
}

// ---- linear form ----------------------------------------------------------------------------------
class LinearFormIntegrator {
public:
    virtual ~LinearFormIntegrator() = default;
};
class DomainLFIntegrator : public LinearFormIntegrator {
public:
    explicit DomainLFIntegrator(Coefficient &f) : Q(&f) {}
    Coefficient *Q;
};

class LinearForm : public Vector {
public:
    explicit LinearForm(FiniteElementSpace *f) : Vector(f->GetVSize()), fes_(f) {}
    void AddDomainIntegrator(LinearFormIntegrator *lfi) { integs_.emplace_back(lfi); }
    void Assemble()
    {
        std::shared_ptr<DeviceSpace> &cached = fes_->LinearFormDevice();
        if (!cached) cached = std::make_shared<DeviceSpace>(*fes_, Array<int>(), false);
        DeviceSpace &dev = *cached;
        const int dim = fes_->GetMesh()->Dimension();
        int nq = 0;
        const std::vector<double> xyz = dev.Points(CDFEM_RULE_LINEARFORM, dim, fes_->GetNE(), nq);
        std::vector<double> fq(xyz.size() / dim, 0.0);
        for (auto &li : integs_) {
            auto *d = dynamic_cast<DomainLFIntegrator *>(li.get());
            if (!d) throw std::invalid_argument("LinearForm: only DomainLFIntegrator is supported");
            const std::vector<double> s = Sample(*d->Q, xyz, dim, nq);
            for (size_t i = 0; i < s.size(); ++i) fq[i] += s[i];
        }
        check(cdfem_lf_assemble(dev.ctx(), fq.data(), GetData(), CDFEM_HOST), dev.ctx(), "cdfem_lf_assemble");
    }

private:
    FiniteElementSpace *fes_;
    std::vector<std::unique_ptr<LinearFormIntegrator>> integs_;
};
using ParLinearForm = LinearForm;

// ---- grid function ----------------------------------------------------------------------------
namespace detail {
// GLL nodes on [0,1] (H1 default basis, GaussLobatto) and the Lagrange basis through them
inline std::vector<double> gll_nodes(int p)
{
    // interior nodes = roots of P_p'; Newton with (1-t^2) P_p' = p (P_{p-1} - t P_p) and the
    // Legendre equation (1-t^2) P_p'' = 2 t P_p' - p (p+1) P_p
    std::vector<double> x((size_t)p + 1);
    x[0] = 0.0;
    x[(size_t)p] = 1.0;
    for (int i = 1; i < p; ++i) {
        double t = -std::cos(M_PI * i / p);
        for (int it = 0; it < 100; ++it) {
            double P0 = 1.0, P1 = t;
            for (int k = 2; k <= p; ++k) {
                const double P2 = ((2 * k - 1) * t * P1 - (k - 1) * P0) / k;
                P0 = P1;
                P1 = P2;
            }
            const double dP = p * (P0 - t * P1) / (1.0 - t * t);
            const double d2P = (2.0 * t * dP - p * (p + 1.0) * P1) / (1.0 - t * t);
            const double dt = dP / d2P;
            t -= dt;
            if (std::fabs(dt) < 1e-16) break;
        }
        x[(size_t)i] = 0.5 * (t + 1.0);
    }
    return x;
}
inline double lagrange(const std::vector<double> &nodes, int i, double t)
{
    double v = 1.0;
    for (size_t k = 0; k < nodes.size(); ++k)
        if ((int)k != i) v *= (t - nodes[k]) / (nodes[(size_t)i] - nodes[k]);
    return v;
}
inline void gauss_legendre01(int n, std::vector<double> &x, std::vector<double> &w)
{
    x.resize((size_t)n);
    w.resize((size_t)n);
    for (int i = 0; i < n; ++i) {
        double t = std::cos(M_PI * (i + 0.75) / (n + 0.5)), dP = 1.0;
        for (int it = 0; it < 100; ++it) {
            double P0 = 1.0, P1 = t;
            for (int k = 2; k <= n; ++k) {
                const double P2 = ((2 * k - 1) * t * P1 - (k - 1) * P0) / k;
                P0 = P1;
                P1 = P2;
            }
            dP = n * (t * P1 - P0) / (t * t - 1.0);
            const double dt = P1 / dP;
            t -= dt;
            if (std::fabs(dt) < 1e-16) break;
        }
        x[(size_t)i] = 0.5 * (1.0 - t);
        w[(size_t)i] = 1.0 / ((1.0 - t * t) * dP * dP);  // (2 / ((1-t^2) P'^2)) / 2
    }
}
}  // namespace detail

class GridFunction : public Vector {
public:
    explicit GridFunction(FiniteElementSpace *f) : Vector(f->GetVSize()), fes_(f) {}
    GridFunction &operator=(double v)
    {
        Vector::operator=(v);
        return *this;
    }
    GridFunction &operator=(const Vector &v)
    {
        Vector::operator=(v);
        return *this;
    }
    FiniteElementSpace *FESpace() const { return fes_; }

    // nodal interpolation (GLL nodal basis: dof value = coefficient at the node)
    void ProjectCoefficient(Coefficient &q) { Project(q, nullptr); }
    void ProjectBdrCoefficient(Coefficient &q, const Array<int> &attr) { Project(q, &attr); }

    // ||u_h - u||_L2 with a tensor Gauss rule of order max(2, 2p+3) (or irs[SQUARE/CUBE])
    double ComputeL2Error(Coefficient &exact, const IntegrationRule *irs[] = nullptr) const
    {
        return L2(&exact, irs, false);
    }
    double ComputeL2Norm(Coefficient &exact, const IntegrationRule *irs[] = nullptr) const
    {
        return L2(&exact, irs, true);
    }

private:
    void Project(Coefficient &q, const Array<int> *attr)
    {
        const int dim = fes_->GetMesh()->Dimension();
        const std::vector<double> &X = fes_->DofCoordinates();
        ElementTransformation T;
        IntegrationPoint ip;
        for (int i = 0; i < Size(); ++i) {
            if (attr && !fes_->OnMarkedBoundary(i, *attr, dim)) continue;
            T.SetPoint(dim, &X[(size_t)i * dim]);
            (*this)[i] = q.Eval(T, ip);
        }
    }
    // simplices: collapsed Gauss with n = p + 3 points per direction (exact to degree 2p + 6 - dim
    // >= the driver's max(2, 2p + 3) in 2D), the product's nodal basis
    double L2Simplex(Coefficient *exact, bool exact_only) const
    {
        const int dim = fes_->GetMesh()->Dimension(), p = fes_->GetOrder(), nd = fes_->NumElementDofs();
        const int nq = cdfem_simplex_rule(dim, p + 3, nullptr, nullptr);
        std::vector<double> xi((size_t)nq * dim), w(nq), phi((size_t)nq * nd);
        cdfem_simplex_rule(dim, p + 3, xi.data(), w.data());
        check(cdfem_simplex_basis(dim, p, nq, xi.data(), phi.data(), nullptr), nullptr, "cdfem_simplex_basis");
        const std::vector<double> &V = fes_->ElementVertices();
        const std::vector<int32_t> &D = fes_->ElementDofs();
        ElementTransformation T;
        IntegrationPoint ip;
        double err2 = 0.0;
        for (int e = 0; e < fes_->GetNE(); ++e) {
            const double *ev = &V[(size_t)e * (dim + 1) * dim];
            double J[3][3] = {};
            for (int k = 0; k < dim; ++k)
                for (int m = 0; m < dim; ++m) J[k][m] = ev[(m + 1) * dim + k] - ev[k];
            const double det = dim == 3 ? J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                                              J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                                              J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0])
                                        : J[0][0] * J[1][1] - J[0][1] * J[1][0];
            for (int q = 0; q < nq; ++q) {
                double X[3] = {0, 0, 0};
                for (int k = 0; k < dim; ++k) {
                    X[k] = ev[k];
                    for (int m = 0; m < dim; ++m) X[k] += J[k][m] * xi[(size_t)q * dim + m];
                }
                double uh = 0.0;
                if (!exact_only)
                    for (int l = 0; l < nd; ++l) uh += phi[(size_t)q * nd + l] * (*this)[D[(size_t)e * nd + l]];
                T.ElementNo = e;
                T.SetPoint(dim, X);
                const double u = exact->Eval(T, ip);
                err2 += w[q] * std::fabs(det) * (uh - u) * (uh - u);
            }
        }
        return std::sqrt(err2);
    }
    double L2(Coefficient *exact, const IntegrationRule *irs[], bool exact_only) const
    {
        if (fes_->Simplex()) return L2Simplex(exact, exact_only);
        const int dim = fes_->GetMesh()->Dimension(), p = fes_->GetOrder(), d1 = p + 1;
        const int geom = dim == 3 ? Geometry::CUBE : Geometry::SQUARE;
        const int order = (irs && irs[geom]) ? irs[geom]->GetOrder() : std::max(2, 2 * p + 3);
        const int nq1 = order / 2 + 1;
        std::vector<double> qx, qw;
        detail::gauss_legendre01(nq1, qx, qw);
        const std::vector<double> nodes = detail::gll_nodes(p);
        std::vector<double> B((size_t)nq1 * d1), G((size_t)nq1 * 2);  // basis at points; vertex hat fns
        for (int q = 0; q < nq1; ++q)
            for (int i = 0; i < d1; ++i) B[(size_t)q * d1 + i] = detail::lagrange(nodes, i, qx[(size_t)q]);
        const int nv = 1 << dim, nd = dim == 3 ? d1 * d1 * d1 : d1 * d1;
        const int nq = dim == 3 ? nq1 * nq1 * nq1 : nq1 * nq1;
        const std::vector<double> &V = fes_->ElementVertices();
        const std::vector<int32_t> &D = fes_->ElementDofs();
        ElementTransformation T;
        IntegrationPoint ip;
        double err2 = 0.0;
        for (int e = 0; e < fes_->GetNE(); ++e) {
            const double *ev = &V[(size_t)e * nv * dim];
            const int32_t *ed = &D[(size_t)e * nd];
            for (int q = 0; q < nq; ++q) {
                const int qi[3] = {q % nq1, (q / nq1) % nq1, q / (nq1 * nq1)};
                double r[3] = {0, 0, 0}, w = 1.0;
                for (int k = 0; k < dim; ++k) {
                    r[k] = qx[(size_t)qi[k]];
                    w *= qw[(size_t)qi[k]];
                }
                // multilinear map and its Jacobian
                double X[3] = {0, 0, 0}, J[3][3] = {};
                for (int v = 0; v < nv; ++v) {
                    double phi = 1.0, dphi[3] = {1, 1, 1};
                    for (int k = 0; k < dim; ++k) {
                        const int b = (v >> k) & 1;
                        const double f = b ? r[k] : 1.0 - r[k], df = b ? 1.0 : -1.0;
                        phi *= f;
                        for (int l = 0; l < dim; ++l) dphi[l] *= (l == k) ? df : f;
                    }
                    for (int k = 0; k < dim; ++k) {
                        X[k] += phi * ev[v * dim + k];
                        for (int l = 0; l < dim; ++l) J[k][l] += dphi[l] * ev[v * dim + k];
                    }
                }
                const double det = dim == 3 ? J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                                                  J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                                                  J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0])
                                            : J[0][0] * J[1][1] - J[0][1] * J[1][0];
                double uh = 0.0;
                if (!exact_only)
                    for (int l = 0; l < nd; ++l) {
                        const int li[3] = {l % d1, (l / d1) % d1, l / (d1 * d1)};
                        double phi = 1.0;
                        for (int k = 0; k < dim; ++k) phi *= B[(size_t)qi[k] * d1 + li[k]];
                        uh += phi * (*this)[ed[l]];
                    }
                T.ElementNo = e;
                T.SetPoint(dim, X);
                const double u = exact->Eval(T, ip);
                err2 += w * std::fabs(det) * (uh - u) * (uh - u);
            }
        }
        return std::sqrt(err2);
    }
    FiniteElementSpace *fes_;
};
using ParGridFunction = GridFunction;

// ||u||_L2 over the mesh (p = 2 only); the geometry is multilinear, so an order-1 space suffices
inline double ComputeGlobalLpNorm(double p, Coefficient &exact, Mesh &mesh, const IntegrationRule *irs[])
{
    if (p != 2.0) throw std::invalid_argument("ComputeGlobalLpNorm: only p = 2");
    H1_FECollection fec(mesh.FromFile() ? 2 : 1, mesh.Dimension());  // simplex rule n = p + 3 >= 5
    FiniteElementSpace fes(&mesh, &fec);
    GridFunction z(&fes);
    return z.ComputeL2Norm(exact, irs);
}

// ---- Krylov solvers ---------------------------------------------------------------------------
class Solver : public Operator {
public:
    using Operator::Operator;
    virtual void SetOperator(const Operator &op) = 0;
};

// MFEM's Jacobi smoother as a preconditioner marker: the solve uses the operator's exact PA
// diagonal (ess rows 1) on the device
class OperatorJacobiSmoother : public Solver {
public:
    OperatorJacobiSmoother() = default;
    void SetOperator(const Operator &) override {}
    void Mult(const Vector &, Vector &) const override
    {
        throw std::logic_error("OperatorJacobiSmoother is applied inside the device solver");
    }
};

// PETSc's PCILU (zero fill, natural ordering) as a preconditioner marker: "-pc_type bjacobi
// -sub_pc_type ilu" (Input/petsc_circle.opts:6-8) on one rank, or "-pc_type ilu".  Factored once per
// operator on the device (ilu_kernels.hip) and applied inside the device GMRES.
class ILUPreconditioner : public Solver {
public:
    ILUPreconditioner() = default;
    void SetOperator(const Operator &) override {}
    void Mult(const Vector &, Vector &) const override
    {
        throw std::logic_error("ILUPreconditioner is applied inside the device solver");
    }
};

class IterativeSolver : public Solver {
public:
    void SetRelTol(double r) { rel_tol = r; }
    void SetAbsTol(double a) { abs_tol = a; }
    void SetMaxIter(int m) { max_iter = m; }
    void SetPrintLevel(int l) { print_level = l; }
    void SetOperator(const Operator &op) override
    {
        oper = dynamic_cast<const ConstrainedPAOperator *>(&op);
        if (!oper) throw std::invalid_argument("solver operator must come from BilinearForm::FormLinearSystem");
        height = width = op.Height();
    }
    void SetPreconditioner(Solver &pc)
    {
        pc_kind = dynamic_cast<OperatorJacobiSmoother *>(&pc) ? CDFEM_PC_JACOBI
                : dynamic_cast<ILUPreconditioner *>(&pc)     ? CDFEM_PC_ILU
                                                              : CDFEM_PC_NONE;
    }
    bool GetConverged() const { return converged; }
    int GetNumIterations() const { return final_iter; }
    double GetFinalNorm() const { return final_norm; }
    double GetSolveSeconds() const { return seconds; }

protected:
    void Run(int method, int restart, const Vector &b, Vector &x) const
    {
        if (!oper) throw std::logic_error("SetOperator was not called");
        cdfem_solver_params prm{};
        prm.method = method;
        prm.pc = pc_kind;
        prm.max_iter = max_iter;
        prm.restart = restart;
        prm.rel_tol = rel_tol;
        prm.abs_tol = abs_tol;
        prm.check_every = 0;
        prm.print_level = print_level;
        cdfem_solver_result res{};
        x.SetSize(b.Size());
        cdfem_ctx *c = oper->Form()->ctx();
        const int rc = cdfem_solve(c, &prm, b.GetData(), x.GetData(), CDFEM_HOST, &res);
        if (rc != CDFEM_OK && rc != CDFEM_ERR_NOT_CONVERGED) check(rc, c, "cdfem_solve");
        converged = res.converged != 0;
        final_iter = res.iterations;
        final_norm = res.final_norm;
        seconds = res.seconds;
        if (print_level > 0)
            std::printf("   Iterations: %d  final norm: %.6e  (initial %.6e)  %s\n", final_iter, final_norm,
                        res.initial_norm, converged ? "converged" : "NOT converged");
    }
    const ConstrainedPAOperator *oper = nullptr;
    double rel_tol = 0.0, abs_tol = 0.0;
    int max_iter = 10, print_level = -1;
    int pc_kind = CDFEM_PC_NONE;
    mutable bool converged = false;
    mutable int final_iter = 0;
    mutable double final_norm = 0.0, seconds = 0.0;
};

// MFEM CGSolver semantics (mesh_recession_handler.cpp:270-276): (r,z) <= max(nom0 rel^2, abs^2).
// MFEM's tolerances are on the norm; cdfem_solve takes them as norms too.
class CGSolver : public IterativeSolver {
public:
    void Mult(const Vector &b, Vector &x) const override { Run(CDFEM_CG, 0, b, x); }
};

// GMRES with PETSc KSPGMRES semantics (left preconditioning, classical Gram-Schmidt)
class GMRESSolver : public IterativeSolver {
public:
    void SetKDim(int m) { kdim = m; }
    void Mult(const Vector &b, Vector &x) const override { Run(CDFEM_GMRES, kdim, b, x); }

private:
    int kdim = 30;
};

// ---- PETSc-named front end (linear_convection_diffusion_2D.cpp:268-282, :364-375) --------------
// MFEMInitializePetsc reads the same option keys the reference's Input/petsc.opts sets:
// -ksp_type {gmres, cg}, -ksp_rtol, -ksp_atol, -ksp_max_it, -ksp_gmres_restart, -pc_type
// {jacobi, none, ilu, bjacobi with -sub_pc_type ilu (-sub_ksp_type preonly)}.  Defaults are PETSc's (gmres, restart 30, rtol 1e-5, atol 1e-50, max_it 1e4,
// pc jacobi for the reference's runs is set by the file).
struct PetscOptionsStore {
    std::map<std::string, std::string> kv;
    std::string Get(const std::string &k, const std::string &def) const
    {
        auto it = kv.find(k);
        return it == kv.end() ? def : it->second;
    }
};
inline PetscOptionsStore &PetscOptions()
{
    static PetscOptionsStore s;
    return s;
}

inline void MFEMInitializePetsc(int * = nullptr, char *** = nullptr, const char *rc_file = nullptr,
                                const char * = nullptr)
{
    if (!rc_file) return;
    std::ifstream in(rc_file);
    if (!in) throw std::runtime_error(std::string("cannot open PETSc options file ") + rc_file);
    std::string line;
    while (std::getline(in, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        std::istringstream ss(line);
        std::string key, val;
        if (!(ss >> key)) continue;
        ss >> val;
        PetscOptions().kv[key] = val;
    }
}
inline void MFEMFinalizePetsc() {}

class PetscParMatrix : public Operator {
public:
    PetscParMatrix(int /*comm*/, const Operator *A, Operator::Type = PETSC_MATAIJ)
        : Operator(A->Height(), A->Width()), A_(A) {}
    void Mult(const Vector &x, Vector &y) const override { A_->Mult(x, y); }
    const Operator *Inner() const { return A_; }

private:
    const Operator *A_;
};

class PetscLinearSolver : public Solver {
public:
    explicit PetscLinearSolver(const PetscParMatrix &A, const std::string & = "")
    {
        const PetscOptionsStore &o = PetscOptions();
        const std::string type = o.Get("-ksp_type", "gmres");
        if (type == "cg") solver_ = std::make_unique<CGSolver>();
        else if (type == "gmres") {
            auto g = std::make_unique<GMRESSolver>();
            g->SetKDim(std::stoi(o.Get("-ksp_gmres_restart", "30")));
            solver_ = std::move(g);
        } else
            throw std::invalid_argument("unsupported -ksp_type " + type);
        solver_->SetRelTol(std::stod(o.Get("-ksp_rtol", "1e-5")));
        solver_->SetAbsTol(std::stod(o.Get("-ksp_atol", "1e-50")));
        solver_->SetMaxIter(std::stoi(o.Get("-ksp_max_it", "10000")));
        const std::string pc = o.Get("-pc_type", "jacobi");
        if (pc == "jacobi") {
            solver_->SetPreconditioner(jac_);
        } else if (pc == "ilu" || pc == "bjacobi") {
            // one rank: block Jacobi has a single block, solved by its sub-PC (preonly + ILU)
            const std::string sub = pc == "ilu" ? "ilu" : o.Get("-sub_pc_type", "ilu");
            const std::string subksp = o.Get("-sub_ksp_type", "preonly");
            if (sub != "ilu" || subksp != "preonly")
                throw std::invalid_argument("unsupported block-Jacobi sub solver " + subksp + "/" + sub);
            solver_->SetPreconditioner(ilu_);
        } else if (pc != "none") {
            throw std::invalid_argument("unsupported -pc_type " + pc);
        }
        SetOperator(A);
    }
    void SetOperator(const Operator &op) override
    {
        const auto *pm = dynamic_cast<const PetscParMatrix *>(&op);
        solver_->SetOperator(pm ? *pm->Inner() : op);
        height = width = op.Height();
    }
    void SetPrintLevel(int l) { solver_->SetPrintLevel(l); }
    void Mult(const Vector &b, Vector &x) const override { solver_->Mult(b, x); }
    bool GetConverged() const { return solver_->GetConverged(); }
    int GetNumIterations() const { return solver_->GetNumIterations(); }
    double GetFinalNorm() const { return solver_->GetFinalNorm(); }
    double GetSolveSeconds() const { return solver_->GetSolveSeconds(); }

private:
    std::unique_ptr<IterativeSolver> solver_;
    OperatorJacobiSmoother jac_;
    ILUPreconditioner ilu_;
};

}  // namespace mfem
}  // namespace cdfem
