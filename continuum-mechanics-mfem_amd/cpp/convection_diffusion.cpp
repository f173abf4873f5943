// convection_diffusion — steady convection-diffusion-reaction MMS solve through the MFEM-shaped
// host API (cdfem_mfem.hpp via mfem.hpp) on the MI355X kernels, one MPI rank per GPU.
//
// The main() below is the reference driver's own sequence, myapps/convection_diffusion/
// linear_convection_diffusion_2D.cpp:238-446, with its call forms unchanged: Mpi::Init / Hypre::Init
// / Mpi::WorldRank, OptionsParser, MFEMInitializePetsc(options file), Device("cpu"),
// make_unique<Mesh>(file, 1, 1) + UniformRefinement, make_unique<ParMesh>(MPI_COMM_WORLD, *mesh),
// MFEM_VERIFY, ParFiniteElementSpace::GlobalTrueVSize, GetEssentialTrueDofs, the three domain
// integrators, ParLinearForm, ProjectBdrCoefficient, FormLinearSystem, Ah.As<HypreParMatrix>(),
// PetscParMatrix(MPI_COMM_WORLD, A, PETSC_MATAIJ), PetscLinearSolver, RecoverFEMSolution,
// ComputeL2Error / ComputeGlobalLpNorm.  What differs: configuration from the command line instead
// of YAML (out of scope), a generated box when no mesh file is given, the 3D extension of
// the MMS (sin(l pi z) factor), and no ParaView / CSV output.  -mms radial runs the
// circle variant instead (linear_convection_diffusion_2D_circle.cpp: u = (r^2-1) cos 2 pi r on the
// unit disk, ValidateUnitCircleMesh, :122-215).
//
//   mpirun -np N convection_diffusion [-d dim] [-n elems | -mesh file.msh] [-p order] [-rs levels]
//       [-rp levels] [-k kappa] [-s reaction] [-c cx,cy,cz] [-m n,m,l] [-mms sin|radial]
//       [-opts petsc.opts] [-pl level]
// Output (rank 0, stdout, one "key value" per line): dofs, ranks, iterations, converged, final_norm,
// l2_abs, l2_rel, solve_seconds.  Exit code 3 on error (as the reference drivers, :435-442).
#include <cmath>
#include <cstdio>
#include <fstream>
#include <memory>
#include <string>

#include "mfem.hpp"

using namespace std;
using namespace mfem;

namespace {

struct Params {
    int dim = 2, n = 16, order = 2, rs = 0, rp = 0, print_level = 0;
    double kappa = 0.1, reaction = 1.0, c[3] = {1.0, -2.0, 0.5};
    int modes[3] = {3, 3, 3};
    string opts, mesh, cstr, mstr, mms = "sin";
};

// the circle variant's radial MMS, linear_convection_diffusion_2D_circle.cpp:140-215:
// u = (r^2 - 1) cos(2 pi r), f = -kappa Lap u + c . grad u + s u with the r -> 0 limits
constexpr double kAlpha = 2.0 * M_PI;
constexpr double kSmallR = 1.0e-12;
double ExactU(double r) { return (r * r - 1.0) * std::cos(kAlpha * r); }
double ExactU_r(double r) { return 2.0 * r * std::cos(kAlpha * r) - kAlpha * (r * r - 1.0) * std::sin(kAlpha * r); }
double ExactU_rr(double r)
{
    return 2.0 * std::cos(kAlpha * r) - 4.0 * kAlpha * r * std::sin(kAlpha * r) -
           kAlpha * kAlpha * (r * r - 1.0) * std::cos(kAlpha * r);
}
double ExactLaplacian(double r) { return r > kSmallR ? ExactU_rr(r) + ExactU_r(r) / r : 2.0 * (2.0 + kAlpha * kAlpha); }

class RadialExactCoefficient : public Coefficient {
public:
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        return ExactU(std::sqrt(x[0] * x[0] + x[1] * x[1]));
    }
};

class RadialForcingCoefficient : public Coefficient {
public:
    explicit RadialForcingCoefficient(const Params &p) : p_(p) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const double r = std::sqrt(x[0] * x[0] + x[1] * x[1]);
        double ux = 0.0, uy = 0.0;
        if (r > kSmallR) {
            const double radial_scale = ExactU_r(r) / r;
            ux = radial_scale * x[0];
            uy = radial_scale * x[1];
        }
        return -p_.kappa * ExactLaplacian(r) + p_.c[0] * ux + p_.c[1] * uy + p_.reaction * ExactU(r);
    }

private:
    const Params &p_;
};

// _circle.cpp:122-138
void ValidateUnitCircleMesh(const ParMesh &pmesh, const double tol)
{
    double local_rmax = 0.0;
    for (int i = 0; i < pmesh.GetNV(); i++) {
        const double *v = pmesh.GetVertex(i);
        local_rmax = std::max(local_rmax, std::sqrt(v[0] * v[0] + v[1] * v[1]));
    }
    double global_rmax = 0.0;
    MPI_Allreduce(&local_rmax, &global_rmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    MFEM_VERIFY(std::abs(global_rmax - 1.0) <= tol,
                "Expected unit-circle mesh (max radius near 1). Found max radius " << global_rmax << ".");
}

// u = sin(n pi x) sin(m pi y) [sin(l pi z)]  (:159-175)
class ExactSolutionCoefficient : public Coefficient {
public:
    ExactSolutionCoefficient(int dim, const int *m) : dim_(dim), m_{m[0], m[1], m[2]} {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        double u = std::sin(m_[0] * M_PI * x[0]) * std::sin(m_[1] * M_PI * x[1]);
        if (dim_ == 3) u *= std::sin(m_[2] * M_PI * x[2]);
        return u;
    }

private:
    int dim_;
    int m_[3];
};

// f = -kappa Lap u + c . grad u + s u for the product of sines (:177-215 and its 3D extension)
class ForcingCoefficient : public Coefficient {
public:
    explicit ForcingCoefficient(const Params &p) : p_(p) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const int d = p_.dim;
        double s[3] = {1, 1, 1}, c[3] = {0, 0, 0}, k2 = 0.0;
        for (int i = 0; i < d; ++i) {
            const double a = p_.modes[i] * M_PI;
            s[i] = std::sin(a * x[i]);
            c[i] = a * std::cos(a * x[i]);
            k2 += a * a;
        }
        const double u = s[0] * s[1] * s[2];
        double conv = 0.0;
        for (int i = 0; i < d; ++i) {
            double g = c[i];
            for (int j = 0; j < d; ++j)
                if (j != i) g *= s[j];
            conv += p_.c[i] * g;
        }
        return p_.kappa * k2 * u + conv + p_.reaction * u;
    }

private:
    const Params &p_;
};

}  // namespace

int main(int argc, char *argv[])
{
    Mpi::Init(argc, argv);
    Hypre::Init();
    const int myid = Mpi::WorldRank();

    Params prm;
    OptionsParser args(argc, argv);
    args.AddOption(&prm.dim, "-d", "--dim", "Dimension of the generated box (2 or 3).");
    args.AddOption(&prm.n, "-n", "--elems", "Elements per direction of the generated box.");
    args.AddOption(&prm.mesh, "-mesh", "--mesh", "gmsh v2.2 mesh file (replaces the box).");
    args.AddOption(&prm.order, "-p", "--order", "H1 order.");
    args.AddOption(&prm.rs, "-rs", "--serial-ref-levels", "Uniform refinements before the partition.");
    args.AddOption(&prm.rp, "-rp", "--par-ref-levels", "Uniform refinements after the partition.");
    args.AddOption(&prm.kappa, "-k", "--kappa", "Diffusion coefficient.");
    args.AddOption(&prm.reaction, "-s", "--reaction", "Reaction coefficient.");
    args.AddOption(&prm.cstr, "-c", "--convection", "Velocity cx,cy[,cz].");
    args.AddOption(&prm.mstr, "-m", "--modes", "MMS modes n,m[,l].");
    args.AddOption(&prm.mms, "-mms", "--mms", "Manufactured solution: sin (the square driver) or radial "
                                              "(the circle driver, 2D unit disk).");
    args.AddOption(&prm.opts, "-opts", "--petsc-options", "PETSc options file.");
    args.AddOption(&prm.print_level, "-pl", "--print-level", "Solver print level.");
    args.Parse();
    if (!args.Good()) {
        if (myid == 0) args.PrintUsage(cerr);
        return 1;
    }
    if (!prm.cstr.empty()) std::sscanf(prm.cstr.c_str(), "%lf,%lf,%lf", &prm.c[0], &prm.c[1], &prm.c[2]);
    if (!prm.mstr.empty()) std::sscanf(prm.mstr.c_str(), "%d,%d,%d", &prm.modes[0], &prm.modes[1], &prm.modes[2]);

    // :268-282, options file (the reference's default path; its values when the file is absent)
    const char *petsc_file_to_use = DriverPetscOptionsFile(prm.opts);
    MFEMInitializePetsc(&argc, &argv, petsc_file_to_use, NULL);

    int exit_code = 0;
    try {
        if (prm.dim != 2 && prm.dim != 3) throw invalid_argument("-d must be 2 or 3");
        const bool radial = prm.mms == "radial";
        if (!radial && prm.mms != "sin") throw invalid_argument("-mms must be sin or radial");
        if (radial && prm.dim != 2) throw invalid_argument("-mms radial is the 2D circle problem");
        Device device("cpu");
        if (myid == 0 && prm.print_level > 0) device.Print(cerr);

        unique_ptr<Mesh> mesh = !prm.mesh.empty() ? make_unique<Mesh>(prm.mesh.c_str(), 1, 1)
                                : prm.dim == 2 ? make_unique<Mesh>(Mesh::MakeCartesian2D(prm.n, prm.n, Element::QUADRILATERAL))
                                               : make_unique<Mesh>(Mesh::MakeCartesian3D(prm.n, prm.n, prm.n, Element::HEXAHEDRON));
        if (mesh->Dimension() != prm.dim) throw runtime_error("-d does not match the mesh file's dimension");
        for (int l = 0; l < prm.rs; l++) mesh->UniformRefinement();

        unique_ptr<ParMesh> pmesh = make_unique<ParMesh>(MPI_COMM_WORLD, *mesh);
        mesh.reset();
        for (int l = 0; l < prm.rp; l++) pmesh->UniformRefinement();

        MFEM_VERIFY(pmesh->bdr_attributes.Size() > 0, "Mesh must define boundary attributes.");
        if (radial) ValidateUnitCircleMesh(*pmesh, 1.0e-8);

        H1_FECollection fec(prm.order, prm.dim);
        ParFiniteElementSpace fespace(pmesh.get(), &fec);
        const HYPRE_BigInt global_true_dofs = fespace.GlobalTrueVSize();

        Array<int> ess_bdr(pmesh->bdr_attributes.Max());
        ess_bdr = 1;
        Array<int> ess_tdof_list;
        fespace.GetEssentialTrueDofs(ess_bdr, ess_tdof_list);

        ExactSolutionCoefficient sin_exact(prm.dim, prm.modes);
        ForcingCoefficient sin_forcing(prm);
        RadialExactCoefficient radial_exact;
        RadialForcingCoefficient radial_forcing(prm);
        Coefficient &exact_coeff = radial ? static_cast<Coefficient &>(radial_exact) : sin_exact;
        Coefficient &forcing_coeff = radial ? static_cast<Coefficient &>(radial_forcing) : sin_forcing;
        Vector c_vec(prm.dim);
        for (int i = 0; i < prm.dim; ++i) c_vec[i] = prm.c[i];
        VectorConstantCoefficient convection_coeff(c_vec);
        ConstantCoefficient kappa_coeff(prm.kappa);
        ConstantCoefficient reaction_coeff(prm.reaction);

        ParBilinearForm a(&fespace);
        a.AddDomainIntegrator(new DiffusionIntegrator(kappa_coeff));
        a.AddDomainIntegrator(new ConvectionIntegrator(convection_coeff));
        a.AddDomainIntegrator(new MassIntegrator(reaction_coeff));
        a.Assemble();

        ParLinearForm b(&fespace);
        b.AddDomainIntegrator(new DomainLFIntegrator(forcing_coeff));
        b.Assemble();

        ParGridFunction u(&fespace);
        u = 0.0;
        u.ProjectBdrCoefficient(exact_coeff, ess_bdr);

        OperatorHandle Ah(Operator::Hypre_ParCSR);
        Vector X, B;
        a.FormLinearSystem(ess_tdof_list, u, b, Ah, X, B);

        int iterations = 0;
        bool converged = true;
        double final_norm = 0.0, seconds = 0.0;
        const int true_size = fespace.TrueVSize();
        const bool all_essential = (ess_tdof_list.Size() == true_size);
        if (!all_essential) {
            HypreParMatrix *A_true = Ah.As<HypreParMatrix>();
            MFEM_VERIFY(A_true != nullptr, "Expected HypreParMatrix from FormLinearSystem.");

            PetscParMatrix A_petsc(MPI_COMM_WORLD, A_true, Operator::PETSC_MATAIJ);
            PetscLinearSolver solver(A_petsc);
            solver.SetPrintLevel(prm.print_level);
            solver.Mult(B, X);
            iterations = solver.GetNumIterations();
            final_norm = solver.GetFinalNorm();
            seconds = solver.GetSolveSeconds();
            converged = solver.GetConverged();
            MFEM_VERIFY(solver.GetConverged(), "PETSc solver did not converge. Iterations="
                                                   << solver.GetNumIterations() << ", residual=" << solver.GetFinalNorm());
        }

        a.RecoverFEMSolution(X, b, u);

        const int order_quad = std::max(2, 2 * prm.order + 3);
        const IntegrationRule *irs[Geometry::NumGeom];
        for (int g = 0; g < Geometry::NumGeom; g++) irs[g] = &IntRules.Get(g, order_quad);

        const double abs_l2 = u.ComputeL2Error(exact_coeff, irs);
        const double exact_l2 = ComputeGlobalLpNorm(2, exact_coeff, *pmesh, irs);
        const double rel_l2 = (exact_l2 > 1.0e-14) ? abs_l2 / exact_l2 : 0.0;

        if (myid == 0)
            std::printf("dofs %lld\nranks %d\niterations %d\nconverged %d\nfinal_norm %.17g\nl2_abs %.17g\n"
                        "l2_rel %.17g\nsolve_seconds %.6g\n",
                        (long long)global_true_dofs, Mpi::WorldSize(), iterations, converged ? 1 : 0, final_norm,
                        abs_l2, rel_l2, seconds);
    } catch (const exception &e) {
        if (myid == 0) cerr << "Error: " << e.what() << endl;
        exit_code = 3;
    }

    MFEMFinalizePetsc();
    return exit_code;
}
